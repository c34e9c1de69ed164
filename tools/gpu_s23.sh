bash tools/gpu_session.sh \
 "fusedtest|300|python -u -m pytest tests/test_conv_f32_gpu.py -k 'bwd_fused or many_tiles' -x -q --timeout 200 --timeout-method thread" \
 "layers|200|python tools/conv_f32_bench.py 3232 10 bwd" \
 "bench|200|python bench.py --also_bf16 0" \
 "bench1|200|python bench.py --also_bf16 0" \
 "torso|300|python -u -m pytest tests/test_conv_f32_gpu.py tests/test_learner_headline_gpu.py -x -q --timeout 300 --timeout-method thread" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof23 -o run -- python3 bench.py --also_bf16 0 --steps 20 --warmup 3"
