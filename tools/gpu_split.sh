#!/bin/bash
# SPLIT-plan session: the SPLIT / segmented-traceback / robustness GPU tests, then configs 2 and 4
# and the per-band timelines (tools/split_stats.py, debug build tools/bin/libstats.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
  -k "split or seg or robust or config2 or probe or golden_large or t16 or flavours" > gpurun_out/pytest_split.log 2>&1 \
  || { tail -40 gpurun_out/pytest_split.log; exit 1; }
tail -2 gpurun_out/pytest_split.log
timeout -k 10 300 python tools/bench_configs.py --only 2,4 > gpurun_out/configs.jsonl 2>&1 || { tail -30 gpurun_out/configs.jsonl; exit 1; }
cat gpurun_out/configs.jsonl
timeout -k 10 150 python tools/split_stats.py sw ${SPLIT_RS:-1 2 4} > gpurun_out/split_sw.txt 2>&1 || { tail -20 gpurun_out/split_sw.txt; exit 1; }
timeout -k 10 150 python tools/split_stats.py lg ${SPLIT_RS:-1 2 4} > gpurun_out/split_lg.txt 2>&1 || { tail -20 gpurun_out/split_lg.txt; exit 1; }
grep -v "^   band" gpurun_out/split_sw.txt gpurun_out/split_lg.txt
