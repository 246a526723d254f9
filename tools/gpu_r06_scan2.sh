#!/bin/bash
# Round 6: alphabet-scan grid size -- pipelined headline kernel trace per grid (scan share, gaps) and steps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for G in 2048 256 64; do
  rm -rf gpurun_out/scan2_$G
  SEQALIB_SCAN_GRID=$G timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/scan2_$G -o run -- python3 bench.py --no-cpu --configs none --dropin-pairs 0 --latency-reps 0 --e2e-steps 1 --serial-steps 1 --out gpurun_out/scan2_$G.json > gpurun_out/scan2_$G.log 2>&1 || { tail -5 gpurun_out/scan2_$G.log; exit 1; }
  python3 tools/pipe_trace.py gpurun_out/scan2_$G --fill fill_so2 > gpurun_out/scan2_$G.pipe.json
  python3 -c "
import json; d=json.load(open('gpurun_out/scan2_$G.pipe.json')); b=json.load(open('gpurun_out/scan2_$G.json'))
rows=d['rows'][2:11]
print('grid $G share', d['scan_share_of_kernel_time'], 'scan_ms', [r['scan_ms'] for r in rows], 'gap_us', [r['gap_us'] for r in rows], 'bench', b['value'], b['ms_per_step'])"
done
SEQALIB_SCAN_GRID=256 timeout -k 10 400 python3 -u tools/fill_sweep.py --sizes "" --variants "base;SEQALIB_SCAN_GRID=256;SEQALIB_SCAN_GRID=64" --rounds 3 --steps 10 2>&1 | grep variant
