"""A/B of few-pair (SPLIT) fills: configs 2 and 4 of tools/bench_configs.py on the library named by
$SEQALIB_HIP_LIB (default: the shipped one).  One JSON line per config.
    SEQALIB_HIP_LIB=seqalib_amd/lib/ab/libg4.so python3 tools/ab_split.py"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "tools"))
os.environ.setdefault("SEQALIB_KERNEL_TIMING", "1")
import torch
import seqalib_amd as sa
from bench_configs import measure
eng = sa.Engine(0)
dev = torch.device("cuda", 0)
lib = os.path.basename(os.environ.get("SEQALIB_HIP_LIB", "libseqalib_hip.so"))
for line in measure(sa, torch, eng, dev, set(sys.argv[1].split(",")) if len(sys.argv) > 1 else {"2", "4"}, 16):
    line.pop("cpu_reference", None)
    print(json.dumps({"lib": lib, **line}), flush=True)
