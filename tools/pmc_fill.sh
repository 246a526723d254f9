#!/bin/bash
# Per-dispatch PMC table of the headline fill: one-pair T16 kernel (SEQALIB_X2=0) vs the two-pair
# packed kernel (SEQALIB_X2=1), one rocprofv3 --pmc pass per counter group (tools/pmc_fill_groups.txt;
# counters this rocprofv3 does not list are dropped from a group first).  Summary:
# gpurun_out/pmc_fill_summary.txt (copied to profiles/ by hand).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
ARGS="--pairs ${PAIRS:-10000} --steps 1 --warmup 1 --no-cpu --e2e-steps 0 --serial-steps 0 --dropin-pairs 0"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  keep=""
  for c in $grp; do grep -q -w "$c" gpurun_out/counters_list.txt && keep="$keep $c"; done
  for x2 in 0 1; do
    rm -rf gpurun_out/pmcf_${i}_$x2
    echo "[pmc] pass $i x2=$x2:$keep"
    SEQALIB_X2=$x2 timeout -s KILL 180 rocprofv3 --pmc $keep --kernel-trace --output-format csv \
      -d gpurun_out/pmcf_${i}_$x2 -o run -- python3 bench.py $ARGS > gpurun_out/pmcf_${i}_$x2.log 2>&1 \
      || { echo "pass $i x2=$x2 failed"; tail -5 gpurun_out/pmcf_${i}_$x2.log; exit 1; }
  done
done < tools/pmc_fill_groups.txt
python3 - <<'PY' > gpurun_out/pmc_fill_summary.txt
import csv, glob, collections
rows = collections.defaultdict(dict)
for f in sorted(glob.glob("gpurun_out/pmcf_*_*/**/*counter_collection.csv", recursive=True)):
    x2 = f.split("pmcf_")[1].split("/")[0].split("_")[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", r.get("KernelName", ""))
        if "fill" not in name: continue
        key = r.get("Dispatch_Id", r.get("Correlation_Id", ""))
        acc[key][r.get("Counter_Name", "")] += float(r.get("Counter_Value", 0))
        acc[key]["_name"] = 0
    # the last big dispatch (the timed step)
    big = [v for v in acc.values() if len(v) > 1]
    if not big: continue
    v = big[-1]
    for k, val in v.items():
        if not k.startswith("_"): rows[x2][k] = val
print("# tools/pmc_fill.sh: 10,000 x 4096^2 SW headline batch, the timed step's fill dispatch, rocprofv3 --pmc (one pass per group)")
print("# SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in quad-cycles (MI355X_MICROARCH.md); x2=0 one pair per wave (T16 CMAX, R=32), x2=1 two pairs per wave (VOP3P, R=16)")
keys = sorted(set(rows.get("0", {})) | set(rows.get("1", {})))
print(f"{'counter':32s} {'one-pair (x2=0)':>18s} {'two-pair (x2=1)':>18s} {'ratio':>8s}")
for k in keys:
    a, b = rows.get("0", {}).get(k), rows.get("1", {}).get(k)
    ratio = f"{b / a:.3f}" if a and b else ""
    print(f"{k:32s} {a if a is not None else float('nan'):18.4g} {b if b is not None else float('nan'):18.4g} {ratio:>8s}")
PY
cat gpurun_out/pmc_fill_summary.txt
