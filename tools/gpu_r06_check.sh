#!/bin/bash
# Round 6: full GPU suite and the default bench line after a change.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-check}
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gputest_$TAG.txt 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/gputest_$TAG.txt | head; tail -30 gpurun_out/gputest_$TAG.txt; exit 1; }
tail -1 gpurun_out/gputest_$TAG.txt
timeout -k 10 600 python bench.py --out gpurun_out/bench_$TAG.json > gpurun_out/bench_$TAG.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_$TAG.json'))
print(d['value'], d['ms_per_step'], d['serial_ms_per_step'], d['e2e_ms_per_step'], d.get('e2e_ms_each'), d['fill_kernel_ms'], d['roofline']['frac'], d['parity'])
print([(c['config'], c.get('gcups'), c.get('fill_kernel_ms'), c.get('ms_per_step')) for c in d['configs']])
print(d['dropin_e2e']['ms_each'])"
