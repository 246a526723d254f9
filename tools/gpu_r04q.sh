#!/bin/bash
# round 4: end-cell candidate statistics, DC parity (capped int32 sweep grid), HB / MM per-kernel times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/so4_stats.py 10000 > gpurun_out/so4_stats.txt 2>&1 || { tail -20 gpurun_out/so4_stats.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/so4_stats.txt
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu \
  -k "hirschberg or myers or dc or endcell" > gpurun_out/gputest_dc.txt 2>&1 || { tail -30 gpurun_out/gputest_dc.txt; exit 1; }
tail -3 gpurun_out/gputest_dc.txt
bash tools/gpu_r04p.sh
