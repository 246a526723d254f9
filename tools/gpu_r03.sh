#!/bin/bash
# Round-3 GPU session: suite -> bench -> configs 2/4 -> SPLIT timelines.  Each GPU step has its
# own limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "[r03] pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
echo "[r03] bench $(date +%T)"
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
echo "[r03] configs $(date +%T)"
timeout -k 10 300 python tools/bench_configs.py --only 2,4 > gpurun_out/configs.jsonl 2>&1 || { tail -30 gpurun_out/configs.jsonl; exit 1; }
cat gpurun_out/configs.jsonl
echo "[r03] split stats $(date +%T)"
timeout -k 10 150 python tools/split_stats.py sw 1 2 4 > gpurun_out/split_sw.txt 2>&1 || { tail -20 gpurun_out/split_sw.txt; exit 1; }
timeout -k 10 150 python tools/split_stats.py lg 1 2 4 > gpurun_out/split_lg.txt 2>&1 || { tail -20 gpurun_out/split_lg.txt; exit 1; }
tail -12 gpurun_out/split_sw.txt
echo "[r03] done $(date +%T)"
