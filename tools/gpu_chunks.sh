set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/chunks.txt
for g in 1 2 4; do
  SEQALIB_HOST_CHUNKS=$g timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 --serial-steps 2 --e2e-steps 3 --dropin-pairs 10000 --dropin-reps 3 > gpurun_out/chunks_$g.log 2>&1 || { tail -5 gpurun_out/chunks_$g.log; exit 1; }
  tail -1 gpurun_out/chunks_$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($g, {k: d[k] for k in ('ms_per_step','e2e_ms_per_step','serial_ms_per_step')}, d['dropin_e2e']['ms_each'])" | tee -a gpurun_out/chunks.txt
done
