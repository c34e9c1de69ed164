# Stage-head backward variants, full fp32 bench each (profiles/experiments.md)
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_f32_gpu.py > gpurun_out/exp_tests.log 2>&1
echo "conv f32 tests: $(tail -1 gpurun_out/exp_tests.log)"
for v in "1:" "0:" "0:0" "0:012"; do
  sc=${v%%:*}; ga=${v#*:}
  SA_F32_POOL_SCATTER=$sc SA_F32_POOL_GATHER=$ga timeout -k 10 150 python bench.py --also_bf16 0 --steps 20 --warmup 5 > gpurun_out/exp1_${sc}_$ga.log 2>&1
  echo "scatter=$sc gather=$ga $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/exp1_${sc}_$ga.log)"
done
