#!/bin/bash
# Plan sweep + counters (experiments; not part of the driver's contract).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/sweep.txt
for plan in ${PLANS:-"16,4" "16,2" "16,1" "8,8" "8,4"}; do
  SEQALIB_PLAN=$plan timeout -k 10 300 python bench.py --pairs ${PAIRS:-8192} --steps 3 --warmup 1 --no-cpu > gpurun_out/sweep_$plan.log 2>&1 || { echo "plan $plan failed"; tail -5 gpurun_out/sweep_$plan.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep_$plan.log').read().strip().splitlines()[-1]); print('$plan', d['value'], d['fill_ms'], d['traceback_ms'], d['roofline']['frac'])" >> gpurun_out/sweep.txt
done
cat gpurun_out/sweep.txt
if [ -n "$PMC" ]; then
  i=0
  while read -r grp; do
    [ -z "$grp" ] && continue; i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmcx_$i -o run -- python3 bench.py --pairs 2048 --steps 1 --warmup 1 --no-cpu > gpurun_out/pmcx_$i.log 2>&1 || echo "pmc pass $i failed"
  done < "$PMC"
fi
