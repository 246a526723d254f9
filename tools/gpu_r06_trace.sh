#!/bin/bash
# Round 6: kernel trace of the pipelined headline legs only (timeline per step, tools/pipe_trace.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/trace_hl
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_hl -o run -- python3 bench.py --no-cpu --configs none --dropin-pairs 0 --latency-reps 0 --e2e-steps 1 --serial-steps 1 --out gpurun_out/trace_hl.json > gpurun_out/trace_hl.log 2>&1 || { tail -5 gpurun_out/trace_hl.log; exit 1; }
python3 tools/pipe_trace.py gpurun_out/trace_hl --fill fill_so2 > gpurun_out/trace_hl_pipe.json
python3 - <<'PY'
import csv, glob
ev = []
for f in glob.glob('gpurun_out/trace_hl/**/*kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:60]))
ev.sort()
fills = [e for e in ev if 'fill_so2' in e[2]]
# the last 4 timed steps: every kernel between fill k start and fill k+1 start
for k in range(len(fills) - 5, len(fills) - 1):
    t0, t1 = fills[k][0], fills[k + 1][0]
    print('--- step', k, 'fill-to-fill', round((t1 - t0) / 1e6, 3), 'ms')
    for s, e, n in ev:
        if t0 <= s < t1:
            print('  %8.3f %8.3f  %s' % ((s - t0) / 1e6, (e - s) / 1e6, n))
PY
