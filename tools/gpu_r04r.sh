#!/bin/bash
# round 4: DC parity + HB / MM per-kernel times (block-aggregated classify, multi-split midpoint kernels)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_dropin_cpp.py -x -q --timeout 120 --timeout-method thread -m gpu \
  -k "hirschberg or myers or dc or Hirschberg or Myers" > gpurun_out/gputest_dc.txt 2>&1 || { tail -30 gpurun_out/gputest_dc.txt; exit 1; }
tail -3 gpurun_out/gputest_dc.txt
bash tools/gpu_r04p.sh
