#!/bin/bash
# round 4: score-only traceback with 8 lanes per pair (SEQALIB_TB_LP=8) -- parity, then per-kernel
# times of the headline step and config 3 at LP = 4 / 8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SEQALIB_TB_LP=8 timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -m gpu \
  > gpurun_out/gputest_lp8.txt 2>&1 || { tail -30 gpurun_out/gputest_lp8.txt; exit 1; }
tail -1 gpurun_out/gputest_lp8.txt
for lp in 4 8 4 8; do
  for shape in "--len 4096" "--len 1024"; do
    rm -rf gpurun_out/lp
    SEQALIB_TB_LP=$lp timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lp -o run -- python3 tools/headline_once.py --calls 3 $shape > gpurun_out/lp.log 2>&1 || { tail -20 gpurun_out/lp.log; exit 1; }
    python3 - "$lp" "$shape" <<'PY'
import csv, glob, sys
f = glob.glob("gpurun_out/lp/**/*kernel_stats.csv", recursive=True)[0]
out = []
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("traceback_so4", "fill_so", "endcell_so")):
        out.append(f"{r['Name'].split('(')[0].replace('void sa::', '')} {float(r['AverageNs']) / 1e3:.1f}us")
print("LP", sys.argv[1], sys.argv[2], " | ".join(out))
PY
  done
done
