#!/bin/bash
# Round 6: column segments for the score-only NW band units (one pair per wave), 10,000 x 1024^2 and 4096^2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for L in 1024 4096; do
timeout -k 10 400 python3 -u tools/fill_sweep.py --algo 1 --sizes "" --len $L --variants "base;SEQALIB_SO_SEGS=4;SEQALIB_SO_SEGS=6;SEQALIB_SO_SEGS=8" --rounds 3 --steps 10 > gpurun_out/segs_nw_$L.jsonl 2>&1 || { tail -5 gpurun_out/segs_nw_$L.jsonl; exit 1; }
grep variant gpurun_out/segs_nw_$L.jsonl | sed "s/{/{\"len\": $L, \"algo\": \"nw\", /"
done
