#!/bin/bash
# End-cell replay per-wave phase cycles (debug stats build) at two batch sizes.
set -o pipefail
mkdir -p gpurun_out
for P in 4000 10000; do
  timeout -k 10 240 python3 -u tools/so4_stats.py $P > gpurun_out/ecstats_$P.txt 2>&1 || exit $?
done
