#!/bin/bash
# 16-bit linear-space sweeps: DC parity + generic tests, tools/bench_dc.py with and without Dc16
# (SEQALIB_DC16=0), then the SPLIT session (tools/gpu_split.sh).  Each GPU step has its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "hirschberg or myers or dc_ or generic or golden" --timeout 120 --timeout-method thread > gpurun_out/dc_tests.log 2>&1 || { echo dc tests failed; tail -30 gpurun_out/dc_tests.log; exit 1; }
tail -2 gpurun_out/dc_tests.log
: > gpurun_out/dc.jsonl
for d16 in 1 0; do for algo in hb mm; do for cfg in "10000 1024" "1000 4096"; do set -- $cfg
  echo "[dc] dc16=$d16 $algo $1 x $2 $(date +%T)"
  SEQALIB_DC16=$d16 timeout -k 10 200 python tools/bench_dc.py --algo $algo --pairs $1 --len $2 --cpu-pairs 0 > gpurun_out/dc_run.log 2>&1 || { echo bench failed; tail -20 gpurun_out/dc_run.log; exit 1; }
  grep '^{' gpurun_out/dc_run.log | sed "s/^{/{\"dc16\": $d16, /" >> gpurun_out/dc.jsonl
done; done; done
cat gpurun_out/dc.jsonl
bash tools/gpu_split.sh
