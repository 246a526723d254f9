#!/bin/bash
# round 4: chunk wave maxima (default) vs the commit before them (libprev) -- same box, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in default prev default prev; do
  lib=seqalib_amd/lib/libseqalib_hip.so; [ $v = prev ] && lib=seqalib_amd/lib/ab/libprev.so
  SEQALIB_HIP_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu --dropin-pairs 0 --configs '' \
    --latency-reps 0 --e2e-steps 0 > gpurun_out/bench_$v.log 2>&1 || { tail -20 gpurun_out/bench_$v.log; exit 1; }
  echo "$v $(grep '^{' gpurun_out/bench_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["fill_kernel_ms"], d["endcell_ms"], d["traceback_ms"], d["parity"][:60])')"
done
