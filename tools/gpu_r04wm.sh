#!/bin/bash
# round 4: chunk wave maxima in the score-only snapshots + two-level end-cell scan -- parity of the
# score-only paths, then kernel times of one headline step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_so.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -m gpu \
  > gpurun_out/gputest_wm.txt 2>&1 || { tail -30 gpurun_out/gputest_wm.txt; exit 1; }
tail -1 gpurun_out/gputest_wm.txt
rm -rf gpurun_out/ecw
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ecw -o run -- python3 tools/headline_once.py --calls 3 > gpurun_out/ecw.log 2>&1 || { tail -20 gpurun_out/ecw.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/ecw/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("endcell", "traceback_so4", "fill_so")):
        print(f"{r['Name'][:50]:50s} {r['Calls']:>3s} calls {float(r['AverageNs']) / 1e3:9.1f} us avg")
PY
