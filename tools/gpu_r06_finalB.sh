#!/bin/bash
# Round 6 final, part B: the default bench line, the same command under rocprofv3 --kernel-trace
# --stats, and the config-5 strong-scaling line at N = 1.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --out gpurun_out/bench_r06_final.json > gpurun_out/bench_r06_final.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench_r06_final.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_r06_final.json'))
print(d['value'], d['ms_per_step'], d['serial_ms_per_step'], d['e2e_ms_per_step'], d['fill_kernel_ms'], d['roofline']['frac'], d['parity'])
print(d['dropin_e2e']['ms_each'])"
rm -rf gpurun_out/rocprof_bench
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rocprof_bench -o run -- python3 bench.py --out gpurun_out/bench_r06_final_rocprof.json > gpurun_out/bench_r06_final_rocprof.log 2>&1 || { echo ROCPROF_FAILED; tail -20 gpurun_out/bench_r06_final_rocprof.log; exit 1; }
head -8 gpurun_out/rocprof_bench/run_kernel_stats.csv
timeout -k 10 600 python bench.py --total-pairs 100000 --len 2048 --steps 5 --warmup 1 --no-cpu --dropin-pairs 0 --latency-reps 0 --configs none --e2e-steps 1 --serial-steps 1 --parity-ops 8 --out gpurun_out/bench_config5_r06_final.json > gpurun_out/bench_config5_r06_final.log 2>&1 || { echo C5_FAILED; tail -30 gpurun_out/bench_config5_r06_final.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_config5_r06_final.json')); print('config5', d['value'], d['ms_per_step'], d['scaling'], d['parity'])"
