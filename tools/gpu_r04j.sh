#!/bin/bash
# round 4: SPLIT hand-off granule A/B (configs 2 and 4)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab_split.jsonl
for lib in seqalib_amd/lib/ab/libg16.so seqalib_amd/lib/ab/libg32.so seqalib_amd/lib/ab/libg16.so seqalib_amd/lib/ab/libg32.so; do
  if [ -n "$lib" ]; then export SEQALIB_HIP_LIB=$PWD/$lib; else unset SEQALIB_HIP_LIB; fi
  timeout -k 10 200 python3 tools/ab_split.py 2,4 >> gpurun_out/ab_split.jsonl 2> gpurun_out/ab_split.err || { tail -20 gpurun_out/ab_split.err; exit 1; }
done
python3 -c "
import json
for l in open('gpurun_out/ab_split.jsonl'):
    d = json.loads(l); print(d['lib'], d['config'], d['workload'][:40], 'call', d.get('ms_per_call'), 'fill', d['fill_ms'], 'kernel', d.get('fill_kernel_ms'), d['parity'][:12])
"
