set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --dropin-pairs 0 --e2e-steps 0 --serial-steps 1 > gpurun_out/bench_so1.json 2> gpurun_out/bench_so1.err || { echo bench failed; tail -20 gpurun_out/bench_so1.err; exit 1; }
cat gpurun_out/bench_so1.json
SEQALIB_SO=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --dropin-pairs 0 --e2e-steps 0 --serial-steps 1 > gpurun_out/bench_so0.json 2>&1 || { echo bench0 failed; exit 1; }
cat gpurun_out/bench_so0.json
