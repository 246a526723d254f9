#!/bin/bash
# Per-config evidence on the GPU box (BASELINE.json configs 2-5 + the C++ drop-in):
#   1. tools/bench_configs.py (all configs, CPU reference beside them)  -> gpurun_out/configs.jsonl
#   2. rocprofv3 --kernel-trace --stats of the single-pair configs 2 and 4 -> gpurun_out/prof_cfg/
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
make -s -C tests/cpp dropin_bench || exit 1
echo "[configs] bench_configs $(date +%T)"
timeout -k 10 600 python tools/bench_configs.py ${ONLY:+--only $ONLY} > gpurun_out/configs.log 2>&1 || { echo configs failed; tail -20 gpurun_out/configs.log; exit 1; }
grep '^{' gpurun_out/configs.log > gpurun_out/configs.jsonl
cat gpurun_out/configs.jsonl
echo "[configs] rocprofv3 configs 2,4 $(date +%T)"
rm -rf gpurun_out/prof_cfg
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg -o run -- python3 tools/bench_configs.py --only 2,4 > gpurun_out/prof_cfg.log 2>&1 || { echo rocprof failed; tail -20 gpurun_out/prof_cfg.log; exit 1; }
find gpurun_out/prof_cfg -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} gpurun_out/configs_kernel_stats.csv
cut -d, -f1-8 gpurun_out/configs_kernel_stats.csv | head -20
echo "[configs] done $(date +%T)"
