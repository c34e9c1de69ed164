# wgrad slot reduction with 16 loads in flight: tests, bench, kernel trace
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_f32_gpu.py tests/test_determinism_gpu.py > gpurun_out/exp_tests.log 2>&1
echo "tests: $(tail -1 gpurun_out/exp_tests.log)"
timeout -k 10 150 python bench.py --also_bf16 0 --steps 20 --warmup 5 > gpurun_out/exp7.log 2>&1
echo "bench $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/exp7.log)"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fp32d -o run -- python3 bench.py --also_bf16 0 --steps 20 --warmup 3 > gpurun_out/prof_fp32d.log 2>&1
