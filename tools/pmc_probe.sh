#!/bin/bash
# Counter probe of the fill kernel on a reduced batch (separate pass per counter group).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS=${ARGS:---pairs 2048 --steps 1 --warmup 1 --no-cpu}
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
grep -o -E "^\s*(SQ|GRBM|TCC|TCP|SPI)_[A-Z0-9_]+" gpurun_out/counters_list.txt | sort -u > gpurun_out/counters_names.txt || true
for grp in "${GROUPS_PMC[@]:-}"; do :; done
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  echo "[pmc] pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc_$i -o run -- python3 bench.py $ARGS > gpurun_out/pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_$i.log; }
done < "${PMC_GROUPS_FILE:-tools/pmc_groups.txt}"
echo done
