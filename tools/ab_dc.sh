#!/bin/bash
# A/B of linear-space aligner builds and leaf thresholds on one box (tuning tool):
#   VARIANTS="cur hb32" ALGO=hb LEAVES="12 24" bash tools/ab_dc.sh   (libs: seqalib_amd/lib/ab/lib<v>.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ALGO=${ALGO:-hb}
ENVV=$([ "$ALGO" = hb ] && echo SEQALIB_HB_LEAF || echo SEQALIB_MM_LEAF)
for v in $VARIANTS; do for leaf in $LEAVES; do for cfg in "10000 1024" "1000 4096"; do set -- $cfg
  env $ENVV=$leaf SEQALIB_HIP_LIB=seqalib_amd/lib/ab/lib$v.so timeout -k 10 120 python tools/bench_dc.py --algo $ALGO --pairs $1 --len $2 --cpu-pairs 0 > gpurun_out/ab_run.log 2>&1 || { echo bench failed; tail -20 gpurun_out/ab_run.log; exit 1; }
  echo "$ALGO $v leaf=$leaf $1x$2 $(grep '^{' gpurun_out/ab_run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_batch"], "ms", d["gcups"], d["parity"])')" | tee -a gpurun_out/ab_dc.txt
done; done; done
