#!/bin/bash
# Round 6: drop-in end-to-end spread -- tests/cpp/dropin_bench 10,000 x 4096^2, 6 reps, three runs,
# with the host phases (SEQALIB_HOST_TIMING) and the cgroup throttling counters per rep.
set -o pipefail
mkdir -p gpurun_out
cat /sys/fs/cgroup/cpu.max > gpurun_out/dropin_cpu_max.txt 2>&1
for k in 1 2 3; do
  SEQALIB_HOST_TIMING=1 timeout -k 10 300 tests/cpp/dropin_bench 10000 4096 6 > gpurun_out/dropin_$k.json 2> gpurun_out/dropin_$k.err || exit 1
  tail -1 gpurun_out/dropin_$k.json
done
