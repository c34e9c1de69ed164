# Scatter wgrad with 2 pooled rows per tile (96 VGPRs): slot sweep
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_f32_gpu.py -k "stage" > gpurun_out/exp_tests.log 2>&1
echo "tests: $(tail -1 gpurun_out/exp_tests.log)"
for v in 2048 1280 1024; do
  SA_F32_PW_SLOTS=$v timeout -k 10 150 python bench.py --also_bf16 0 --steps 20 --warmup 5 > gpurun_out/exp8_$v.log 2>&1
  echo "pw_slots=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/exp8_$v.log)"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SA_F32_PW_SLOTS=1280 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pw -o run -- python3 bench.py --also_bf16 0 --steps 20 --warmup 3 > gpurun_out/prof_pw.log 2>&1
