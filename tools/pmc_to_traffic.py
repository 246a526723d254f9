#!/usr/bin/env python3
"""Store a tools/pmc_roofline.sh summary as the headline fill's PMC record, the one bench.py
reports (profiles/pmc_traffic.json, keyed by workload; the kernel label guards against reporting a
record of another kernel):
    python3 tools/pmc_to_traffic.py gpurun_out/roofline_final/summary.json sw_so2_r32 "<source>" """
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
summ, label, source = sys.argv[1], sys.argv[2], sys.argv[3]
s = json.load(open(summ))
entry = {"label": label, "kernel": s["kernel"], "hbm_bytes_per_launch": s["hbm_bytes_per_launch"],
         "fetch_bytes": s["fetch_bytes"], "write_bytes": s["write_bytes"], "hbm_basis": s["hbm_basis"],
         "clock_ghz": round(s["clock_ghz"], 4), "valu_wave_instr_per_cell": round(s["valu_wave_instr_per_cell"], 4),
         "wait_inst_frac": round(s["wait_inst_frac"], 4), "kernel_ms_per_pass": s["durations_ms_per_pass"],
         "counters": s["counters"], "source": source}
path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
d = json.load(open(path))
d["sw_batch_10000x4096x4096"] = entry
json.dump(d, open(path, "w"), indent=1)
print(json.dumps({k: entry[k] for k in ("hbm_bytes_per_launch", "clock_ghz", "valu_wave_instr_per_cell", "kernel_ms_per_pass")}))
