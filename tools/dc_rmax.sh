#!/bin/bash
# Tuning probe: rows per lane of the whole-wave DC sweeps (SEQALIB_DC_RMAX), both aligners.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for algo in hb mm; do for rmax in 32 4 2; do for cfg in "10000 1024" "1000 4096"; do set -- $cfg
  SEQALIB_DC_RMAX=$rmax timeout -k 10 120 python tools/bench_dc.py --algo $algo --pairs $1 --len $2 --cpu-pairs 0 > gpurun_out/ab_run.log 2>&1 || { echo bench failed; tail -20 gpurun_out/ab_run.log; exit 1; }
  echo "$algo rmax=$rmax $1x$2 $(grep '^{' gpurun_out/ab_run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_batch"], "ms", d["gcups"], d["parity"])')"
done; done; done
