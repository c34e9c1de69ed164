bash tools/gpu_session.sh \
 "convtest|300|python -u -m pytest tests/test_conv_f32_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "layers|200|python tools/conv_f32_bench.py 3232 10 deep" \
 "bench|200|python bench.py --also_bf16 0" \
 "benchfl0|200|SA_WINO_FL=0 python bench.py --also_bf16 0" \
 "bench1|200|python bench.py --also_bf16 0" \
 "torso|300|python -u -m pytest tests/test_learner_headline_gpu.py tests/test_learner_parity_gpu.py -x -q --timeout 300 --timeout-method thread" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof24 -o run -- python3 bench.py --also_bf16 0 --steps 20 --warmup 3"
