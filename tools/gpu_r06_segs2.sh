#!/bin/bash
# Round 6: column segments per band unit at 2048^2 and 1024^2 (10,000 pairs, pipelined steps, alternating).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for L in 2048 1024; do
timeout -k 10 400 python3 -u tools/fill_sweep.py --sizes "" --len $L --variants "base;SEQALIB_SO_SEGS=3;SEQALIB_SO_SEGS=4;SEQALIB_SO_SEGS=6;SEQALIB_SO_SEGS=8" --rounds 3 --steps 20 > gpurun_out/segs_$L.jsonl 2>&1 || { tail -5 gpurun_out/segs_$L.jsonl; exit 1; }
grep -v amdgpu.ids gpurun_out/segs_$L.jsonl | sed "s/^/$L /"
done
