#!/bin/bash
# Round-3 session: full -m gpu suite, headline bench (no CPU legs), host-API end-to-end timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[c] pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
echo "[c] bench $(date +%T)"
timeout -k 10 300 python bench.py --no-cpu --dropin-pairs 0 > gpurun_out/bench_q.log 2>&1 || { tail -20 gpurun_out/bench_q.log; exit 1; }
tail -1 gpurun_out/bench_q.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step','fill_ms','endcell_traceback_ms','e2e_ms_per_step','serial_ms_per_step','parity')})"
echo "[c] e2e trace $(date +%T)"
rm -rf gpurun_out/prof_e2e
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_e2e -o run -- python3 bench.py --no-cpu --dropin-pairs 0 --steps 1 --warmup 1 --serial-steps 0 --e2e-steps 2 > gpurun_out/prof_e2e.log 2>&1 || { tail -20 gpurun_out/prof_e2e.log; exit 1; }
python3 tools/trace_timeline.py gpurun_out/prof_e2e --last-ms 70 > gpurun_out/e2e_timeline.txt 2>&1
tail -40 gpurun_out/e2e_timeline.txt
echo "[c] dc kernel stats $(date +%T)"
for algo in hb mm; do
  rm -rf gpurun_out/prof_dc_$algo
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dc_$algo -o run -- python3 tools/bench_dc.py --algo $algo --pairs 10000 --len 1024 --cpu-pairs 0 > gpurun_out/prof_dc_$algo.log 2>&1 || { tail -20 gpurun_out/prof_dc_$algo.log; exit 1; }
  grep '^{' gpurun_out/prof_dc_$algo.log | cut -c1-200
done
