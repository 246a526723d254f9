#!/bin/bash
# Round 6: column segments per band unit with the two-pairs-per-wave fill (pipelined headline steps, alternating).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u tools/fill_sweep.py --sizes "" --variants "${SEGS_VARIANTS:-base;SEQALIB_SO_SEGS=1;SEQALIB_SO_SEGS=3;SEQALIB_SO_SEGS=4}" --rounds 3 --steps 10 > gpurun_out/segs_r06.jsonl 2>&1 || { tail -5 gpurun_out/segs_r06.jsonl; exit 1; }
cat gpurun_out/segs_r06.jsonl | grep -v amdgpu.ids
