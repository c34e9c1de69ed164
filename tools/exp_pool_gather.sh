# Stage-head backward variants: pre-pool gradient gathered inside the conv
# kernels for stages 1/2 (stage 0 always scatter), full fp32 bench each
set -e
for ga in "" 2 12; do
  SA_F32_POOL_GATHER=$ga timeout -k 10 150 python bench.py --also_bf16 0 --steps 20 --warmup 5 > gpurun_out/exp5_$ga.log 2>&1
  echo "gather=$ga $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/exp5_$ga.log)"
done
