#!/bin/bash
# round 4: two-per-wave 16-bit HB sweeps -- DC tests, A/B timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[o] dbg + DC tests $(date +%T)"
timeout -k 10 200 python -u tools/dbg_dc16.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_generic.py -x -q --timeout 300 --timeout-method thread -k "hirschberg or myers or dc or Hirschberg or linear" > gpurun_out/pytest_o.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_o.log
[ $rc -eq 0 ] || exit $rc
echo "[o] A/B $(date +%T)"
: > gpurun_out/dc_seg16.jsonl
for algo in hb mm; do
for v in 1 0 1 0; do
  SEQALIB_DC_SEG16=$v timeout -k 10 200 python3 tools/bench_dc.py --algo $algo --pairs 10000 --len 1024 --cpu-pairs 0 > gpurun_out/dc_seg16_$v.log 2>&1 || { tail -20 gpurun_out/dc_seg16_$v.log; exit 1; }
  grep '^{' gpurun_out/dc_seg16_$v.log | sed "s/^{/{\"seg16\": $v, /" >> gpurun_out/dc_seg16.jsonl
done
done
SEQALIB_DC_SEG16=1 timeout -k 10 200 python3 tools/bench_dc.py --algo hb --pairs 1000 --len 4096 --cpu-pairs 0 > gpurun_out/dc_seg16_4k.log 2>&1 && grep '^{' gpurun_out/dc_seg16_4k.log | sed 's/^{/{"seg16": 1, /' >> gpurun_out/dc_seg16.jsonl
cut -c1-200 gpurun_out/dc_seg16.jsonl
