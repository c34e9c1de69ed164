#!/bin/bash
# Occupancy sweep of the fp32 conv forward/dgrad grids (SA_F32_FWD_OCC) and
# the stage-head grid (SA_F32_POOL_OCC): per-layer times and the full bench.
mkdir -p gpurun_out
for occ in 2 3 4; do
  SA_F32_FWD_OCC=$occ timeout -k 10 120 python tools/conv_f32_bench.py 3232 5 deep > gpurun_out/occ_layers_$occ.log 2>&1 || exit 1
  SA_F32_FWD_OCC=$occ SA_F32_POOL_OCC=$occ timeout -k 10 200 python bench.py --steps 20 --warmup 3 --also_bf16 0 > gpurun_out/occ_bench_$occ.log 2>&1 || exit 1
  echo "occ=$occ $(tail -1 gpurun_out/occ_bench_$occ.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  grep -E "fwd|dgrad" gpurun_out/occ_layers_$occ.log | grep -v amdgpu
done
