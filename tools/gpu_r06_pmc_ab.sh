#!/bin/bash
# Round 6: PMC roofline of the headline fill, two pairs per wave (default) and one (SEQALIB_SO2=0).
set -o pipefail
OUT=gpurun_out/roofline_so2 bash tools/pmc_roofline.sh > gpurun_out/pmc_so2.txt 2>&1 || { tail -20 gpurun_out/pmc_so2.txt; exit 1; }
SEQALIB_SO2=0 OUT=gpurun_out/roofline_so1 bash tools/pmc_roofline.sh > gpurun_out/pmc_so1.txt 2>&1 || { tail -20 gpurun_out/pmc_so1.txt; exit 1; }
tail -25 gpurun_out/pmc_so2.txt; echo ======; tail -25 gpurun_out/pmc_so1.txt
