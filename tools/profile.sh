#!/bin/bash
# Headline bench + rocprofv3 evidence, on the GPU box.
#   1. bench.py at its defaults (10,000 x 4096^2 SW, with the CPU baseline)  -> gpurun_out/bench_full.json
#   2. rocprofv3 --kernel-trace --stats of the same command (no CPU leg)      -> gpurun_out/prof_stats/
#   3. rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE (separate passes)   -> gpurun_out/prof_fetch|write/
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
BENCH_ARGS=${BENCH_ARGS:-}
echo "[profile] bench $(date +%T)"
timeout -k 10 900 python bench.py $BENCH_ARGS --out gpurun_out/bench_full.json > gpurun_out/bench_full.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_full.log; exit 1; }
cat gpurun_out/bench_full.json
echo "[profile] kernel-trace --stats $(date +%T)"
rm -rf gpurun_out/prof_stats gpurun_out/prof_fetch gpurun_out/prof_write
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- python3 bench.py $BENCH_ARGS --no-cpu --out gpurun_out/bench_prof.json > gpurun_out/prof_stats.log 2>&1 || { echo stats failed; tail -20 gpurun_out/prof_stats.log; exit 1; }
echo "[profile] pmc FETCH_SIZE $(date +%T)"
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_fetch -o run -- python3 bench.py $BENCH_ARGS --no-cpu --steps 1 --warmup 1 > gpurun_out/prof_fetch.log 2>&1 || { echo fetch failed; tail -20 gpurun_out/prof_fetch.log; exit 1; }
echo "[profile] pmc WRITE_SIZE $(date +%T)"
timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_write -o run -- python3 bench.py $BENCH_ARGS --no-cpu --steps 1 --warmup 1 > gpurun_out/prof_write.log 2>&1 || { echo write failed; tail -20 gpurun_out/prof_write.log; exit 1; }
python3 tools/summarize_profile.py --tag "$TAG" > gpurun_out/profile_summary.txt 2>&1 || { echo summarize failed; cat gpurun_out/profile_summary.txt; exit 1; }
cat gpurun_out/profile_summary.txt
echo "[profile] done $(date +%T)"
