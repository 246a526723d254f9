#!/bin/bash
# Round 6 A/B: the score-only fill with an agent-scope release fence (buffer_wbl2 sc1) before every
# unit's per-unit word and an acquire (buffer_inv sc1) in the final unit (SA_SO2_FENCE build,
# seqalib_amd/lib/ab/libfence.so) -- the cost of publishing a unit's streams to another XCD.
set -o pipefail
B="--steps 10 --warmup 2 --no-cpu --dropin-pairs 0 --latency-reps 0 --configs none --e2e-steps 0 --serial-steps 2 --parity-ops 0"
for k in 1 2; do
  timeout -k 10 300 python3 bench.py $B --out gpurun_out/fence_base_$k.json > /dev/null 2>&1 || exit 1
  SEQALIB_HIP_LIB=seqalib_amd/lib/ab/libfence.so timeout -k 10 300 python3 bench.py $B --out gpurun_out/fence_on_$k.json > /dev/null 2>&1 || exit 1
done
for f in gpurun_out/fence_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['fill_kernel_ms'], d['serial_ms_per_step'], d['parity_exact'])"; done
