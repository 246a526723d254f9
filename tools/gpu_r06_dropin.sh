#!/bin/bash
# Round 6: drop-in end-to-end -- tests/cpp/dropin_bench 10,000 x 4096^2, 6 reps, per-rep host phases
# and page faults: GPU call in chunks of 2,048 / 5,000 pairs (lists of landed chunks beside it) and
# one chunk, with the host buffers kept across calls.
set -o pipefail
mkdir -p gpurun_out
for k in 1 2; do
for cp in 2048 5000 100000; do
  SEQALIB_LIST_CHUNK_PAIRS=$cp SEQALIB_HOST_TIMING=1 timeout -k 10 300 tests/cpp/dropin_bench 10000 4096 6 > gpurun_out/dropin_b${cp}_$k.json 2> gpurun_out/dropin_b${cp}_$k.err || exit 1
  echo $cp; tail -1 gpurun_out/dropin_b${cp}_$k.json | cut -c 150-330
done
done
