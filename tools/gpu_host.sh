#!/bin/bash
# Host-API session: host-API / drop-in / multi-context GPU tests, host phase timing (1 and 2
# chunks), bench with the e2e and drop-in legs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "robust or dropin or host or multi or pipelined or generic" > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -2 gpurun_out/pt.log
for g in 1 2; do
  echo G=$g
  SEQALIB_HOST_CHUNKS=$g SEQALIB_HOST_TIMING=1 timeout -k 10 200 python tools/host_api_timing.py > gpurun_out/hat_$g.log 2>&1 || { tail -5 gpurun_out/hat_$g.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/hat_$g.log
done
timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 --serial-steps 2 --e2e-steps 3 --dropin-pairs 10000 --dropin-reps 3 > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('ms_per_step','e2e_ms_per_step','serial_ms_per_step')}, d['dropin_e2e']['ms_each'])"
