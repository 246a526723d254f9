#!/bin/bash
# Round 6: 8 column segments for the packed fill -- score-only / hand-off tests, then the default bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_so.py tests/test_gpu_handoff.py > gpurun_out/so8_tests.txt 2>&1 || { tail -30 gpurun_out/so8_tests.txt; exit 1; }
tail -2 gpurun_out/so8_tests.txt
timeout -k 10 700 python bench.py --out gpurun_out/bench_r06_c.json > gpurun_out/bench_r06_c.log 2>&1 || { tail -20 gpurun_out/bench_r06_c.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_r06_c.json'))
print(d['value'], d['ms_per_step'], d['serial_ms_per_step'], d['e2e_ms_per_step'], d['fill_kernel_ms'], d['roofline']['frac'], d['parity'])
print([(c['config'], c.get('gcups'), c.get('fill_kernel_ms'), c.get('ms_per_step'), c.get('parity') if isinstance(c.get('parity'), str) else c.get('parity',{}).get('exact')) for c in d['configs']])
print(d['dropin_e2e']['ms_each'])"
