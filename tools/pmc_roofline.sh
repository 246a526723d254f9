#!/bin/bash
# Roofline evidence of the shipped headline fill, one rocprofv3 run per pass
# on tools/headline_once.py (one warm-up call + one measured call):
#   1. --kernel-trace --stats                      -> per-kernel durations
#   2. --pmc FETCH_SIZE      3. --pmc WRITE_SIZE   -> HBM bytes per fill dispatch (separate passes)
#   4. --pmc SQ_* instruction / wave counters + GRBM_GUI_ACTIVE -> VALU per cell, clock
#   5. --pmc SQ_* busy / wait cycles + GRBM_GUI_ACTIVE
# tools/pmc_roofline.py summarises them into gpurun_out/roofline/summary.json (-> profiles/).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/roofline}
rm -rf $OUT && mkdir -p $OUT
RUN="python3 tools/headline_once.py --calls 2"
echo "[roofline] stats $(date +%T)"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $RUN > $OUT/stats.log 2>&1 \
  || { echo stats failed; tail -20 $OUT/stats.log; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
           "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY"; do
  i=$((i+1))
  echo "[roofline] pmc pass $i: $grp $(date +%T)"
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/pmc_$i -o run -- $RUN > $OUT/pmc_$i.log 2>&1 \
    || { echo "pmc pass $i failed"; tail -20 $OUT/pmc_$i.log; exit 1; }
done
python3 tools/pmc_roofline.py $OUT > $OUT/summary.txt || { echo summary failed; cat $OUT/summary.txt; exit 1; }
cat $OUT/summary.txt
