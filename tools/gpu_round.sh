#!/bin/bash
# One GPU session of the round: every -m gpu test, the SPLIT session (configs 2/4, timelines), the
# headline bench without the CPU legs, and the linear-space batches (HB/MM 10,000 x 1024^2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_full.sh || exit 1
echo "[round] bench $(date +%T)"
timeout -k 10 300 python bench.py --no-cpu --dropin-pairs 0 > gpurun_out/bench_quick.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_quick.log; exit 1; }
grep '^{' gpurun_out/bench_quick.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step','fill_ms','endcell_traceback_ms','e2e_ms_per_step','serial_ms_per_step','parity')})"
: > gpurun_out/dc.jsonl
for algo in hb mm; do
  echo "[round] dc $algo $(date +%T)"
  timeout -k 10 200 python tools/bench_dc.py --algo $algo --pairs 10000 --len 1024 --cpu-pairs 0 > gpurun_out/dc_run.log 2>&1 || { echo dc bench failed; tail -20 gpurun_out/dc_run.log; exit 1; }
  grep '^{' gpurun_out/dc_run.log >> gpurun_out/dc.jsonl
done
cat gpurun_out/dc.jsonl
