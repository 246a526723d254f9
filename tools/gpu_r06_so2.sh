#!/bin/bash
# Round 6: two-pairs-per-wave score-only SW fill (sa_fill_so2.hip): GPU parity, then the headline
# A/B against one pair per wave (SEQALIB_SO2=0), alternating.
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_so.py tests/test_gpu_handoff.py > gpurun_out/so2_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/so2_tests.log; exit 1; }
tail -3 gpurun_out/so2_tests.log
B="--steps 10 --warmup 2 --no-cpu --dropin-pairs 0 --latency-reps 0 --configs none --e2e-steps 1 --serial-steps 2 --parity-ops 4"
for k in 1 2; do
  SEQALIB_SO2=0 timeout -k 10 300 python bench.py $B --out gpurun_out/so2_ab_old_$k.json > /dev/null 2>gpurun_out/so2_ab_old_$k.err || exit 1
  timeout -k 10 300 python bench.py $B --out gpurun_out/so2_ab_new_$k.json > /dev/null 2>gpurun_out/so2_ab_new_$k.err || exit 1
done
for f in gpurun_out/so2_ab_*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); r=d['roofline']
print('$f', d['value'], d['ms_per_step'], 'fill_kernel', d['fill_kernel_ms'], 'tb', d['traceback_ms'], 'serial', d['serial_ms_per_step'], 'e2e', d['e2e_ms_per_step'], 'parity', d['parity_exact'])"; done
