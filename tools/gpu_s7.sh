bash tools/gpu_session.sh \
 "tests|500|python -u -m pytest tests/test_conv_f32_gpu.py tests/test_learner_parity_gpu.py -q -m gpu --timeout 300 --timeout-method thread" \
 "bench|200|python bench.py --also_bf16 0" \
 "benchs|200|python bench.py --also_bf16 0 --torso shallow" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --also_bf16 0 --steps 20 --warmup 3"
