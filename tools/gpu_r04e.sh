#!/bin/bash
# round 4: Dc16 steady-chunk park fix (dbg + DC tests + HB/MM A/B), full GPU suite, PMC roofline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[e] dbg_dc16 $(date +%T)"
timeout -k 10 200 python -u tools/dbg_dc16.py > gpurun_out/dbg_dc16.log 2>&1; rc=$?
cat gpurun_out/dbg_dc16.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
echo "[e] dc tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "hirschberg or myers or dc or Hirschberg or Myers" > gpurun_out/pytest_dc.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_dc.log
[ $rc -eq 0 ] || exit $rc
echo "[e] dc A/B $(date +%T)"
: > gpurun_out/dc_ab.jsonl
for park in 1 0; do
  for algo in hb mm; do
    SEQALIB_DC16_PARK=$park timeout -k 10 200 python3 tools/bench_dc.py --algo $algo --pairs 10000 --len 1024 --cpu-pairs 0 > gpurun_out/dc_ab_$algo$park.log 2>&1 || { tail -20 gpurun_out/dc_ab_$algo$park.log; exit 1; }
    grep '^{' gpurun_out/dc_ab_$algo$park.log | sed "s/^{/{\"park\": $park, /" >> gpurun_out/dc_ab.jsonl
  done
done
cut -c1-220 gpurun_out/dc_ab.jsonl
echo "[e] launch count $(date +%T)"
bash tools/launch_count.sh || exit 1
echo "[e] full suite $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -8 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
echo "[e] roofline $(date +%T)"
bash tools/pmc_roofline.sh > gpurun_out/roofline.log 2>&1; rc=$?
tail -40 gpurun_out/roofline.log
exit $rc
