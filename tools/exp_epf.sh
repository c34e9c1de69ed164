# 16-channel forward/dgrad with epilogue-operand prefetch (199 VGPRs: 2 WGs/CU)
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_f32_gpu.py > gpurun_out/exp_tests.log 2>&1
echo "conv f32 tests: $(tail -1 gpurun_out/exp_tests.log)"
SA_F32_FWD_OCC=2 timeout -k 10 300 python tools/conv_f32_bench.py 3232 5 deep > gpurun_out/l_epf.log 2>&1
grep res16 gpurun_out/l_epf.log
SA_F32_FWD_OCC=2 timeout -k 10 150 python bench.py --also_bf16 0 --steps 20 --warmup 5 > gpurun_out/exp6.log 2>&1
echo "bench occ2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/exp6.log)"
