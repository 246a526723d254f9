"""Lane-level simulation of the 16-bit HirschbergSA whole-wave sweep band (hb_band16): the
per-step-branch schedule and the branch-free steady-chunk schedule with the LDS-parked hand-off row
(round 3, not shipped), both against a plain NWScore row.  Both schedules match on random shapes,
so the wrong rows the steady variant produced on the GPU come from its code generation, not its
schedule."""
import numpy as np
# wave simulation of hb_band16 (int arithmetic, no 16-bit), one band, generic vs steady
def nwrow(A, B, G, MA, MI):
    m, n = len(A), len(B)
    H = [j * G for j in range(n + 1)]
    for i in range(1, m + 1):
        prev = H[:]
        H[0] = i * G
        for j in range(1, n + 1):
            s = MA if A[i-1] == B[j-1] else MI
            H[j] = max(prev[j-1] + s, max(prev[j], H[j-1]) + G)
    return H
def sweep(A, B, R, G, MA, MI, steady_on):
    m, n = len(A), len(B)
    BAND = 64 * R
    assert m <= BAND
    tl, rl = (m - 1) // R, (m - 1) % R
    out = [0] * (n + 1)
    lanes = range(64)
    a = [[A[l*R + r] if l*R + r < m else -1 for r in range(R)] for l in lanes]
    Hp = [[(l*R + r + 1) * G for r in range(R)] for l in lanes]
    prev_up = [l * R * G for l in lanes]
    hl = [0] * 64
    sym = [0] * 64
    def load(c0):
        vu = [0]*64; vs = [0]*64
        for l in lanes:
            j = c0 + l
            if j < n: vu[l] = (j + 1) * G; vs[l] = B[j]
        return vu, vs
    def cell(l, up, sy):
        hd, hu = prev_up[l], up
        for r in range(R):
            s = MA if a[l][r] == sy else MI
            h = max(hd + s, max(hu, Hp[l][r]) + G)
            hd = Hp[l][r]; Hp[l][r] = h; hu = h
        prev_up[l] = up
        hl[l] = Hp[l][R - 1]
    vup, vsym = load(0)
    c0 = 0
    while c0 < n + 63:
        nvup, nvsym = load(c0 + 64)
        st = steady_on and c0 >= 63 and c0 + 64 <= n
        steps = 64 if st else min(64, n + 63 - c0)
        park = [0] * 128
        for q in range(steps):
            s_ = c0 + q
            up = [vup[q]] + hl[:63]          # DPP wave_shr:1 with old = readlane(vup, q) for lane 0
            sy = [vsym[q]] + sym[:63]
            sym[:] = sy
            for l in lanes:
                j0 = s_ - l
                if st or (0 <= j0 < n):
                    cell(l, up[l], sy[l])
                    if st:
                        park[(0 if l == tl else 64) + q] = Hp[l][rl]
                    elif l == tl:
                        out[j0 + 1] = Hp[l][rl]
        if st:
            for l in lanes:
                out[c0 - tl + 1 + l] = park[l]
        vup, vsym = nvup, nvsym
        c0 += 64
    out[0] = m * G
    return out
rng = np.random.default_rng(1)
for it in range(30):
    m = int(rng.integers(1, 129)); n = int(rng.integers(1, 400)); R = 2 if m <= 128 else 4
    A = list(rng.integers(0, 4, m)); B = list(rng.integers(0, 4, n))
    ref = nwrow(A, B, -1, 2, -1)
    g = sweep(A, B, R, -1, 2, -1, False)
    s = sweep(A, B, R, -1, 2, -1, True)
    if g != ref or s != ref:
        print("mismatch", m, n, g == ref, s == ref)
print("done")
