#!/bin/bash
# round 4: score-only cell with LDS row profiles (SA_SO_LDSPROF) -- parity, then headline A/B against v_bfe_i32
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu \
  > gpurun_out/gputest_ldsprof.txt 2>&1 || { tail -30 gpurun_out/gputest_ldsprof.txt; exit 1; }
tail -2 gpurun_out/gputest_ldsprof.txt
for v in default bfe default bfe; do
  lib=seqalib_amd/lib/libseqalib_hip.so; [ $v = bfe ] && lib=seqalib_amd/lib/ab/libbfe.so
  SEQALIB_HIP_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu --dropin-pairs 0 --configs '' \
    --latency-reps 0 --e2e-steps 0 > gpurun_out/bench_$v.log 2>&1 || { tail -20 gpurun_out/bench_$v.log; exit 1; }
  echo "$v $(grep '^{' gpurun_out/bench_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["fill_kernel_ms"], d["endcell_ms"], d["traceback_ms"], d["parity"][:60])')"
done
