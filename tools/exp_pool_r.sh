# Stage-0 fused conv+pool tile height / residency sweep (full fp32 bench)
set -e
for v in "3:2" "2:3" "1:4" "2:2"; do
  r=${v%%:*}; o=${v#*:}
  SA_F32_POOL_R=$r SA_F32_POOL_OCC=$o timeout -k 10 150 python bench.py --also_bf16 0 --steps 20 --warmup 5 > gpurun_out/exp4_$r_$o.log 2>&1
  echo "R=$r occ=$o $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/exp4_$r_$o.log)"
done
