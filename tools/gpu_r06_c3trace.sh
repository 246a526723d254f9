#!/bin/bash
# Round 6: kernel timeline of pipelined 10,000 x 1024^2 SW steps (config 3 shape).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/c3trace
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c3trace -o run -- python3 bench.py --len 1024 --steps 20 --no-cpu --configs none --dropin-pairs 0 --latency-reps 0 --e2e-steps 1 --serial-steps 1 --out gpurun_out/c3trace.json > gpurun_out/c3trace.log 2>&1 || { tail -5 gpurun_out/c3trace.log; exit 1; }
python3 - <<'PY'
import csv, glob, json
ev = []
for f in glob.glob('gpurun_out/c3trace/**/*kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:55]))
ev.sort()
fills = [e for e in ev if 'fill_so2' in e[2]]
for k in range(8, 11):
    t0, t1 = fills[k][0], fills[k + 1][0]
    print('--- step', k, 'fill-to-fill', round((t1 - t0) / 1e6, 3), 'ms')
    for s, e, n in ev:
        if t0 <= s < t1:
            print('  %8.3f %8.3f  %s' % ((s - t0) / 1e6, (e - s) / 1e6, n))
d = json.load(open('gpurun_out/c3trace.json'))
print('bench', d['value'], d['ms_per_step'], d['fill_kernel_ms'])
PY
