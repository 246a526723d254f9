#!/bin/bash
# Kernel launches per single-pair drop-in call: rocprofv3 kernel trace of
# tests/cpp/dropin_latency restricted to one call kind; launches / calls from the kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=${REPS:-20}
for kind in nw sw; do
  rm -rf gpurun_out/prof_lc_$kind
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lc_$kind -o run -- tests/cpp/dropin_latency $REPS $kind > gpurun_out/prof_lc_$kind.log 2>&1 || { tail -20 gpurun_out/prof_lc_$kind.log; exit 1; }
  python3 - "$kind" "$REPS" <<'PY'
import csv, glob, sys
kind, reps = sys.argv[1], int(sys.argv[2])
calls = reps if kind == "nw" else max(1, reps // 4)
calls += 1   # the first (untimed) call
f = glob.glob(f"gpurun_out/prof_lc_{kind}/**/*kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
tot = sum(int(r["Calls"]) for r in rows)
print(f"{kind}: {tot} kernel launches over {calls} calls = {tot / calls:.2f} per call")
for r in sorted(rows, key=lambda r: -int(r["Calls"])):
    print(f"   {int(r['Calls']):6d}  {float(r['AverageNs']) / 1e3:9.1f} us  {r['Name'][:110]}")
PY
done
