#!/bin/bash
# Per-dispatch PMC table of the headline fill (10,000 x 4096^2 SW, T16 one pair per wave, R = 32):
# one rocprofv3 --pmc pass per counter group (tools/pmc_fill_groups.txt; counters this rocprofv3
# does not list are dropped from a group first).  Summary (tools/pmc_summary.py):
# gpurun_out/pmc_fill_summary.txt (copied to profiles/ by hand).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
ARGS="--pairs ${PAIRS:-10000} --steps 1 --warmup 1 --no-cpu --e2e-steps 0 --serial-steps 0 --dropin-pairs 0"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  keep=""
  for c in $grp; do grep -q -w "$c" gpurun_out/counters_list.txt && keep="$keep $c"; done
  rm -rf gpurun_out/pmcf_${i}_0
  echo "[pmc] pass $i:$keep"
  timeout -s KILL 180 rocprofv3 --pmc $keep --kernel-trace --output-format csv \
    -d gpurun_out/pmcf_${i}_0 -o run -- python3 bench.py $ARGS > gpurun_out/pmcf_${i}_0.log 2>&1 \
    || { echo "pass $i failed"; tail -5 gpurun_out/pmcf_${i}_0.log; exit 1; }
done < tools/pmc_fill_groups.txt
python3 tools/pmc_summary.py gpurun_out > gpurun_out/pmc_fill_summary.txt
cat gpurun_out/pmc_fill_summary.txt
