#!/bin/bash
# Round 6: branch-free end-cell replay -- SW parity tests, then the replay time by batch size.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_so.py tests/test_gpu_handoff.py > gpurun_out/ec2_tests.txt 2>&1 || { tail -30 gpurun_out/ec2_tests.txt; exit 1; }
tail -3 gpurun_out/ec2_tests.txt
for P in 4000 10000; do
  rm -rf gpurun_out/ec_$P
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ec_$P -o run -- python3 tools/headline_once.py --pairs $P --calls 3 > gpurun_out/ec_$P.log 2>&1 || { tail -5 gpurun_out/ec_$P.log; exit 1; }
  python3 - <<PY
import csv, glob
for f in glob.glob('gpurun_out/ec_$P/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'endcell_so' in r['Name'] or 'fill_so' in r['Name'] or 'traceback_so' in r['Name']:
            print($P, r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
PY
done
