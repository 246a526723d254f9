#!/bin/bash
# Round 6: the packed fill at R = 16 (1024^2 batches): SW and NW against one pair per wave, segment counts.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for A in 0 1; do
timeout -k 10 400 python3 -u tools/fill_sweep.py --algo $A --sizes "" --len 1024 --variants "base;SEQALIB_SO2=0;SEQALIB_SO_SEGS=4;SEQALIB_SO2=0,SEQALIB_SO_SEGS=4" --rounds 3 --steps 20 > gpurun_out/r16_$A.jsonl 2>&1 || { tail -5 gpurun_out/r16_$A.jsonl; exit 1; }
grep -E "variant" gpurun_out/r16_$A.jsonl | sed "s/^/algo$A /"
done
