#!/bin/bash
# Round 6: the alphabet scan behind a running fill -- kernel traces of the pipelined headline with
# one-wave scan workgroups (default) and the round-5 256-thread ones (SEQALIB_SCAN_WG=256), then
# plain bench A/B lines of both.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="--steps 10 --warmup 2 --no-cpu --dropin-pairs 0 --latency-reps 0 --configs none --e2e-steps 0 --serial-steps 0 --parity-ops 0"
for v in 64 256; do
  rm -rf gpurun_out/scan_tr_$v
  SEQALIB_SCAN_WG=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/scan_tr_$v -o run -- python3 bench.py $B > gpurun_out/scan_tr_$v.log 2>&1 || { tail -20 gpurun_out/scan_tr_$v.log; exit 1; }
  python3 tools/pipe_trace.py gpurun_out/scan_tr_$v > gpurun_out/scan_tr_$v.json || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/scan_tr_$v.json')); print('$v', 'scan share', d['scan_share_of_kernel_time'], 'mean gap us', d['mean_gap_us']); [print('  ', r) for r in d['rows'][:4]]"
done
for k in 1 2; do
  for v in 256 64; do
    SEQALIB_SCAN_WG=$v timeout -k 10 300 python3 bench.py $B --out gpurun_out/scan_ab_${v}_$k.json > /dev/null 2>&1 || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/scan_ab_${v}_$k.json')); print('scan_wg $v', d['value'], d['ms_per_step'], d['fill_kernel_ms'])"
  done
done
