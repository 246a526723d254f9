#!/bin/bash
# A/B of engine builds on one box: LIBS="build/libA.so build/libB.so" ROUNDS=2 bash tools/ab.sh [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab.txt
for r in $(seq ${ROUNDS:-2}); do
  for lib in $LIBS; do
    SEQALIB_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --steps ${STEPS:-3} --warmup 1 "$@" > gpurun_out/ab_run.log 2>&1 || { echo "$lib failed"; tail -5 gpurun_out/ab_run.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_run.log').read().strip().splitlines()[-1]); print('$lib', d['value'], d['fill_ms'], d['endcell_traceback_ms'], d['ms_per_step'])" >> gpurun_out/ab.txt
  done
done
cat gpurun_out/ab.txt
