#!/bin/bash
# Round 6: full GPU suite, the default bench line, and the config-5 strong-scaling line at N = 1.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r06}
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gputest_$TAG.txt 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gputest_$TAG.txt; exit 1; }
tail -2 gpurun_out/gputest_$TAG.txt
timeout -k 10 600 python bench.py --out gpurun_out/bench_$TAG.json > gpurun_out/bench_$TAG.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench_$TAG.log; exit 1; }
tail -c 600 gpurun_out/bench_$TAG.json; echo
if [ -n "$CONFIG5" ]; then
timeout -k 10 600 python bench.py --total-pairs 100000 --len 2048 --steps 5 --warmup 1 --no-cpu --dropin-pairs 0 --latency-reps 0 --configs none --e2e-steps 1 --serial-steps 1 --parity-ops 8 --out gpurun_out/bench_config5_$TAG.json > gpurun_out/bench_config5_$TAG.log 2>&1 || { echo C5_FAILED; tail -30 gpurun_out/bench_config5_$TAG.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_config5_$TAG.json')); print('config5', d['value'], d['ms_per_step'], d['scaling'], d['config']['workload'], d['parity'])"
fi
