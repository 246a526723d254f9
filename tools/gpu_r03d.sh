#!/bin/bash
# Round-3 session: DC parity tests + DC batches (steady-chunk 16-bit sweeps), then the host-API
# session (tools/gpu_host.sh).  Each GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/dbg_dc16.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "hirschberg or myers or dc_ or generic or golden" --timeout 120 --timeout-method thread > gpurun_out/dc_tests.log 2>&1 || { echo dc tests failed; tail -30 gpurun_out/dc_tests.log; exit 1; }
tail -2 gpurun_out/dc_tests.log
: > gpurun_out/dc.jsonl
for algo in hb mm; do for cfg in "10000 1024" "1000 4096"; do set -- $cfg
  timeout -k 10 200 python tools/bench_dc.py --algo $algo --pairs $1 --len $2 --cpu-pairs 0 > gpurun_out/dc_run.log 2>&1 || { echo bench failed; tail -20 gpurun_out/dc_run.log; exit 1; }
  grep '^{' gpurun_out/dc_run.log >> gpurun_out/dc.jsonl
done; done
cut -c1-220 gpurun_out/dc.jsonl
bash tools/gpu_host.sh
echo "[d] headline-only rocprof $(date +%T)"
rm -rf gpurun_out/prof_head
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_head -o run -- python3 bench.py --no-cpu --dropin-pairs 0 --steps 5 --warmup 1 --serial-steps 0 --e2e-steps 0 > gpurun_out/prof_head.log 2>&1 || { tail -20 gpurun_out/prof_head.log; exit 1; }
tail -1 gpurun_out/prof_head.log | cut -c1-200
echo "[d] full suite $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
echo "[d] bench $(date +%T)"
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-400
