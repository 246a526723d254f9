#!/usr/bin/env python3
"""VALU issue-bound model of a fill kernel's steady loop (the roofline "peak" of bench.py).

The fill kernel is bound by VALU instruction issue, not HBM (0.25 B/cell) and not MFMA (no
matrix work).  gfx950 issues different opcodes at different rates (profiles/
microbench_valu_issue_r01.txt: 16-bit add/max, mov, f32 add/fma ~0.41 wave-instr/cycle/SIMD;
32-bit max/min/cmp/carry/shift-or/bfe/alignbit ~0.22-0.23), so the ceiling depends on the mix.

This script compiles the fill TU for gfx950, takes the largest basic block of the requested
kernel (the branch-free steady chunk loop: SPP steps x R rows per lane), prices every VALU
instruction at its measured issue rate and reports
    cycles_per_lane_cell = sum(count / rate) / cells_per_lane_in_block   [SIMD cycles / 64 cells]
    peak_gcups = SIMDs * clock * 64 / cycles_per_lane_cell / 1e9
Scalar and memory instructions issue on other units and are not charged.
    python3 tools/issue_model.py [--out profiles/issue_model_r03.json]
"""
import argparse, collections, json, os, re, subprocess, sys, tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RATES_FILES = [os.path.join(ROOT, "profiles", f) for f in ("microbench_valu_issue_r01.txt", "microbench_sdwa_r01.txt")]
SIMDS, CLOCK = 256 * 4, 2.4e9

ALIAS = {"v_mov_b32_dpp": "v_mov_b32_dpp_shr", "v_readlane_b32": "readlane", "v_writelane_b32": "readlane",
         "v_mov_b32": "mov_b32", "v_max_i16": "max_i16", "v_add_u16": "add_u16", "v_alignbit_b32": "alignbit_b32",
         "v_bfe_i32": "v_bfe_u32", "v_addc_co_u32": "addc_only", "v_cndmask_b32": "cndmask_e64_sgpr",
         "v_add_u16_sdwa": "add_u16_sdwa_byte1_sext", "v_sub_u16": "sub_u16_e64_clamp",
         "v_cmp_eq_u32": "cmp_only", "v_cmp_gt_u32": "cmp_only", "v_cmp_le_u32": "cmp_only",
         "v_lshl_add_u64": "v_lshl_add_u32", "v_max3_i32": "v_max3_i32", "v_add_co_u32": "add_co_e64",
         # packed 16-bit forms measured at one rate (profiles/microbench_valu_issue_r01.txt)
         "v_pk_sub_u16": "v_pk_add_u16", "v_pk_max_u16": "v_pk_max_i16",
         # the f16 cell's packed ops: the same cycles per cell as the integer forms
         # (tools/microbench_pk6.hip PK5F vs PK5, profiles/microbench_pk5f_r06.txt)
         "v_pk_add_f16": "v_pk_add_u16", "v_pk_maximum3_f16": "v_pk_max_i16",
         # one-half SDWA conversions: the SDWA rate (profiles/microbench_sdwa_r01.txt)
         "v_cvt_u16_f16_sdwa": "mov_b32_sdwa_preserve", "v_cvt_f16_u16_sdwa": "mov_b32_sdwa_preserve"}

KERNELS = {  # label -> (TU, mangled name, cells per lane in one steady block = SPP * R [* pairs per lane])
    # round 6: the score-only SW fill with two pairs per wave (fill_so2_kernel<R>, sa_fill_so2.hip)
    # (fill_so2_kernel<ALG, R, FK>; FK: the f16 cell, the default for SW at f16-exact scorings)
    "sw_so2f_r32": ("sa_fill_so2.hip", "_ZN2sa15fill_so2_kernelILi0ELi32ELb1EEEvNS_10FillParamsE", 512),   # 8 steps x 32 rows x 2 pairs
    "sw_so2f_r16": ("sa_fill_so2.hip", "_ZN2sa15fill_so2_kernelILi0ELi16ELb1EEEvNS_10FillParamsE", 256),
    "sw_so2_r32": ("sa_fill_so2.hip", "_ZN2sa15fill_so2_kernelILi0ELi32ELb0EEEvNS_10FillParamsE", 512),
    "sw_so2_r16": ("sa_fill_so2.hip", "_ZN2sa15fill_so2_kernelILi0ELi16ELb0EEEvNS_10FillParamsE", 256),
    # round 5: the score-only fills (fill_so_kernel<ALG, R>): SW / NW band units, LG / GG affine
    "sw_so_r32": ("sa_fill_sw.hip", "_ZN2sa14fill_so_kernelILi0ELi32EEEvNS_10FillParamsE", 256),   # 8 steps x 32 rows
    "sw_so_r16": ("sa_fill_sw.hip", "_ZN2sa14fill_so_kernelILi0ELi16EEEvNS_10FillParamsE", 128),
    "nw_so_r16": ("sa_fill_nw.hip", "_ZN2sa14fill_so_kernelILi1ELi16EEEvNS_10FillParamsE", 128),
    "lg_so_r16": ("sa_fill_lg.hip", "_ZN2sa14fill_so_kernelILi2ELi16EEEvNS_10FillParamsE", 64),    # 4 steps x 16 rows
    "gg_so_r16": ("sa_fill_gg.hip", "_ZN2sa14fill_so_kernelILi3ELi16EEEvNS_10FillParamsE", 64),
    # the tagged T16 and int32 fills (records for the traceback)
    "sw_t16c_r32": ("sa_fill_sw.hip", "_ZN2sa11fill_kernelILi0ELi32ELi0ELb1ELb1ELb1ELb1ELb0ELb0EEEvNS_10FillParamsE", 64),
    "nw_t16_r16": ("sa_fill_nw.hip", "_ZN2sa11fill_kernelILi1ELi16ELi0ELb1ELb0ELb1ELb0ELb0ELb0EEEvNS_10FillParamsE", 64),
    "lg_t16c_r16": ("sa_fill_lg.hip", "_ZN2sa11fill_kernelILi2ELi16ELi0ELb1ELb1ELb1ELb1ELb0ELb0EEEvNS_10FillParamsE", 16),
    "gg_t16_r16": ("sa_fill_gg.hip", "_ZN2sa11fill_kernelILi3ELi16ELi0ELb1ELb0ELb1ELb0ELb0ELb0EEEvNS_10FillParamsE", 16),
    "sw_int32_r16": ("sa_fill_sw.hip", "_ZN2sa11fill_kernelILi0ELi16ELi0ELb1ELb1ELb0ELb0ELb0ELb0EEEvNS_10FillParamsE", 64),
}


def rates():
    r = {}
    for f in RATES_FILES:
        if not os.path.exists(f):
            continue
        for line in open(f):
            m = re.match(r"^(\S+)\s+[\d.]+ ms\s+([\d.]+) wave-instr", line)
            if m:
                r.setdefault(m.group(1), float(m.group(2)))
    return r


def rate_of(op, R):
    base = re.sub(r"_e(32|64)$", "", op)
    for k in (op, base, ALIAS.get(op), ALIAS.get(base)):
        if k and k in R:
            return R[k]
    return None


def steady_block(asm, name):
    st = asm.find(name + ":")
    en = asm.find(".Lfunc_end", st)   # not the first s_endpgm: the variant guard returns early
    blocks, cur = [], []
    for line in asm[st:en].split("\n"):
        if re.match(r"^\.LBB|^_Z|^; %bb\.", line):
            blocks.append(cur)
            cur = []
        else:
            t = line.strip()
            if t and not t.startswith(";") and not t.startswith("."):
                cur.append(t.split()[0])
    blocks.append(cur)
    return max(blocks, key=len)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--kernels", default=",".join(KERNELS))
    a = ap.parse_args()
    R = rates()
    out = {"rates_files": [os.path.relpath(f, ROOT) for f in RATES_FILES], "simds": SIMDS, "clock_hz": CLOCK, "kernels": {}}
    cache = {}
    with tempfile.TemporaryDirectory() as td:
        for label in a.kernels.split(","):
            tu, name, cells = KERNELS[label]
            if tu not in cache:
                subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c",
                                os.path.join(ROOT, "seqalib_amd", "csrc", tu), "-o", os.path.join(td, "x.o"),
                                "-save-temps"], cwd=td, check=True, capture_output=True)
                s = [f for f in os.listdir(td) if f.endswith("gfx950.s") and f.startswith(tu[:-4])][0]
                cache[tu] = open(os.path.join(td, s)).read()
            blk = steady_block(cache[tu], name)
            cnt = collections.Counter(blk)
            cyc, valu, elem, unknown = 0.0, 0, 0, {}
            two = "so2" in label   # two pairs per lane: packed ops and v_perm carry two cells' work
            for op, c in cnt.items():
                if not op.startswith("v_"):
                    continue
                valu += c
                elem += c * (2 if (op.startswith("v_pk_") or (two and op.startswith("v_perm"))) else 1)
                r = rate_of(op, R)
                if r is None:
                    unknown[op] = c
                    r = 0.22
                cyc += c / r
            cpc = cyc / cells
            out["kernels"][label] = {
                "kernel": name, "cells_per_lane_in_block": cells, "valu_per_cell": round(valu / cells, 3),
                # lane-element ops: a packed 16-bit op (and, two pairs per lane, a v_perm) does two
                # lanes' work, issuing at half the wave rate -- the quantity the VALU peak counts
                "valu_elem_per_cell": round(elem / cells, 3),
                "cycles_per_lane_cell": round(cpc, 3),
                "peak_gcups": round(SIMDS * CLOCK * 64 / cpc / 1e9, 1),
                "mix": dict(sorted(((k, v) for k, v in cnt.items() if k.startswith("v_")), key=lambda x: -x[1])),
                "unpriced_at_slow_rate": unknown}
            print(f"{label:14s} VALU/cell {valu / cells:6.2f}  cycles/lane-cell {cpc:6.2f}  "
                  f"issue ceiling {SIMDS * CLOCK * 64 / cpc / 1e9:8.1f} GCUPS  unpriced {unknown}")
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
