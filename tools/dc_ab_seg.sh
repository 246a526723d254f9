set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "hirschberg or myers or dc_level" --timeout 120 --timeout-method thread > gpurun_out/dc_tests.log 2>&1 || { echo dc tests failed; tail -30 gpurun_out/dc_tests.log; exit 1; }
tail -1 gpurun_out/dc_tests.log
for algo in mm hb; do for seg in 1 0; do for cfg in "10000 1024" "1000 4096"; do set -- $cfg
SEQALIB_DC_SEG=$seg timeout -k 10 120 python tools/bench_dc.py --algo $algo --pairs $1 --len $2 --cpu-pairs 0 > gpurun_out/ab_run.log 2>&1 || { echo bench failed; tail -20 gpurun_out/ab_run.log; exit 1; }
echo "$algo seg=$seg $1x$2 $(grep '^{' gpurun_out/ab_run.log | cut -c70-200)"
done; done; done
for leaf in 12 16; do SEQALIB_HB_LEAF=$leaf SEQALIB_MM_LEAF=$leaf timeout -k 10 120 python tools/bench_dc.py --algo hb --pairs 10000 --len 1024 --cpu-pairs 0 > gpurun_out/ab_run.log 2>&1 && echo "hb leaf=$leaf $(grep '^{' gpurun_out/ab_run.log | cut -c70-200)"; SEQALIB_MM_LEAF=$leaf timeout -k 10 120 python tools/bench_dc.py --algo mm --pairs 10000 --len 1024 --cpu-pairs 0 > gpurun_out/ab_run.log 2>&1 && echo "mm leaf=$leaf $(grep '^{' gpurun_out/ab_run.log | cut -c70-200)"; done
