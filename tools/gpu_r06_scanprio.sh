#!/bin/bash
# Round 6: pipelined calls' alphabet scan on a highest-priority stream (SEQALIB_SCAN_PRIO) -- the
# pipeline tests, then the kernel-trace scan share and steps either way, then an alternating step A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_handoff.py tests/test_gpu_configs.py tests/test_gpu_robust.py tests/test_gpu_parity.py > gpurun_out/scanprio_tests.log 2>&1 || { tail -20 gpurun_out/scanprio_tests.log; exit 1; }
tail -2 gpurun_out/scanprio_tests.log
for P in 1 0; do
  rm -rf gpurun_out/scanprio_$P
  SEQALIB_SCAN_PRIO=$P timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/scanprio_$P -o run -- python3 bench.py --no-cpu --configs none --dropin-pairs 0 --latency-reps 0 --e2e-steps 1 --serial-steps 1 --out gpurun_out/scanprio_$P.json > gpurun_out/scanprio_$P.log 2>&1 || { tail -5 gpurun_out/scanprio_$P.log; exit 1; }
  python3 tools/pipe_trace.py gpurun_out/scanprio_$P --fill fill_so2 > gpurun_out/scanprio_$P.pipe.json
  python3 -c "
import json; d=json.load(open('gpurun_out/scanprio_$P.pipe.json')); b=json.load(open('gpurun_out/scanprio_$P.json'))
rows=d['rows'][2:11]
print('prio $P share', d['scan_share_of_kernel_time'], 'scan_ms', [r['scan_ms'] for r in rows], 'gap_us', [r['gap_us'] for r in rows], 'bench', b['value'], b['ms_per_step'])"
done
timeout -k 10 400 python3 -u tools/fill_sweep.py --sizes "" --variants "base;SEQALIB_SCAN_PRIO=0" --rounds 3 --steps 10 2>&1 | grep variant
