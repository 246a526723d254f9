"""Merged kernel / memory-copy timeline of the last LAST_MS milliseconds of a rocprofv3 run
(--kernel-trace --memory-copy-trace --output-format csv).  Used to see where an end-to-end host API
call spends its time (uploads, fills, tracebacks, downloads and the gaps between them).

    python tools/trace_timeline.py gpurun_out/prof_e2e [--last-ms 60] [--min-us 20]
"""
import argparse
import csv
import glob
import os


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last-ms", type=float, default=60.0)
    ap.add_argument("--min-us", type=float, default=20.0, help="hide events shorter than this")
    a = ap.parse_args()
    ev = []
    for r in rows(a.dir, "*kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K",
                   r.get("Kernel_Name", "")[:70], r.get("Stream_Id", r.get("Queue_Id", ""))))
    for r in rows(a.dir, "*memory_copy_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C",
                   f'{r.get("Direction", "")} {int(r.get("Size", 0) or 0) / 1e6:.1f} MB', ""))
    if not ev:
        print("no trace rows under", a.dir)
        return
    end = max(e[1] for e in ev)
    t0 = end - int(a.last_ms * 1e6)
    sel = sorted(e for e in ev if e[1] >= t0)
    base = sel[0][0]
    busy_k = []
    print(f"{'start ms':>9s} {'end ms':>9s} {'dur ms':>8s}  kind  what")
    for s, e, k, what, q in sel:
        if k == "K":
            busy_k.append((s, e))
        if (e - s) / 1e3 < a.min_us:
            continue
        print(f"{(s - base) / 1e6:9.3f} {(e - base) / 1e6:9.3f} {(e - s) / 1e6:8.3f}  {k:4s}  {what} {q}")
    # idle gaps of the GPU (no kernel running) longer than 0.1 ms
    busy_k.sort()
    cur = busy_k[0][1]
    gaps = []
    for s, e in busy_k[1:]:
        if s > cur + 100000:
            gaps.append(((cur - base) / 1e6, (s - cur) / 1e6))
        cur = max(cur, e)
    print("kernel-idle gaps > 0.1 ms (at ms, length ms):", [(round(x, 3), round(y, 3)) for x, y in gaps])


if __name__ == "__main__":
    main()
