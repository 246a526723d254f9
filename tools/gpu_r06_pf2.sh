#!/bin/bash
# Round 6: traceback kernel time with and without the walk prefetch (rocprofv3 kernel stats, 3 calls each).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for PF in 1 0 1 0; do
  rm -rf gpurun_out/pf2_$PF
  SEQALIB_TB_PF=$PF timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pf2_$PF -o run -- python3 tools/headline_once.py --calls 3 > gpurun_out/pf2_$PF.log 2>&1 || { tail -5 gpurun_out/pf2_$PF.log; exit 1; }
  python3 - <<PY
import csv, glob
for f in glob.glob('gpurun_out/pf2_$PF/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'traceback_so4' in r['Name']:
            print('PF=$PF', r['Name'][:45], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us', round(float(r['MinNs'])/1e3,1))
PY
done
