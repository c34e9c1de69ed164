# Fused conv+pool for deep stages 1/2 (SA_F32_FUSED_POOL), full fp32 bench each
set -e
for v in 0 01 012; do
  SA_F32_FUSED_POOL=$v timeout -k 10 150 python bench.py --also_bf16 0 --steps 20 --warmup 5 > gpurun_out/exp9_$v.log 2>&1
  echo "fused=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/exp9_$v.log)"
done
