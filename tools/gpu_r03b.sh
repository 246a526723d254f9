#!/bin/bash
# Round-3 measurement session: linear-space batches (Dc16 on/off), SPLIT timelines (configs 2/4),
# rocprofv3 kernel stats of the headline bench, then the PMC fill table.  Each GPU step has its
# own limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/dc.jsonl
for d16 in 1 0; do for algo in hb mm; do for cfg in "10000 1024" "1000 4096"; do set -- $cfg
  echo "[dc] dc16=$d16 $algo $1 x $2 $(date +%T)"
  SEQALIB_DC16=$d16 timeout -k 10 200 python tools/bench_dc.py --algo $algo --pairs $1 --len $2 --cpu-pairs 0 > gpurun_out/dc_run.log 2>&1 || { echo bench failed; tail -20 gpurun_out/dc_run.log; exit 1; }
  grep '^{' gpurun_out/dc_run.log | sed "s/^{/{\"dc16\": $d16, /" >> gpurun_out/dc.jsonl
done; done; done
cat gpurun_out/dc.jsonl
echo "[split] $(date +%T)"
timeout -k 10 150 python tools/split_stats.py sw 1 2 4 > gpurun_out/split_sw.txt 2>&1 || { tail -20 gpurun_out/split_sw.txt; exit 1; }
timeout -k 10 150 python tools/split_stats.py lg 1 2 4 > gpurun_out/split_lg.txt 2>&1 || { tail -20 gpurun_out/split_lg.txt; exit 1; }
grep -v "^   band" gpurun_out/split_sw.txt gpurun_out/split_lg.txt | tail -30
echo "[rocprof] $(date +%T)"
rm -rf gpurun_out/prof_bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --no-cpu --dropin-pairs 0 --steps 5 --warmup 1 > gpurun_out/prof_bench.log 2>&1 || { tail -20 gpurun_out/prof_bench.log; exit 1; }
tail -1 gpurun_out/prof_bench.log | cut -c1-300
echo "[pmc] $(date +%T)"
bash tools/pmc_fill.sh
