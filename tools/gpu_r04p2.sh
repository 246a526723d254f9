#!/bin/bash
# round 4: headline bench (pipelined steps) with fill / traceback stream priorities on (1) and off (0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lp in 1 0 1 0; do
  SEQALIB_STREAM_PRIO=$lp timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu --dropin-pairs 0 --configs '' \
    --latency-reps 0 --e2e-steps 2 > gpurun_out/bench_prio$lp.log 2>&1 || { tail -20 gpurun_out/bench_prio$lp.log; exit 1; }
  echo "PRIO $lp $(grep '^{' gpurun_out/bench_prio$lp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["fill_kernel_ms"], d["endcell_ms"], d["traceback_ms"], d["serial_ms_per_step"], d["e2e_ms_per_step"], d["parity"][:30])')"
done
