bash tools/gpu_session.sh \
 "fwdtest|300|python -u -m pytest tests/test_conv_f32_gpu.py -k 'residual_block_forward or many_tiles or forward' -x -q --timeout 200 --timeout-method thread" \
 "fwdtest3w|300|SA_WINO16_3W=1 python -u -m pytest tests/test_conv_f32_gpu.py -k 'residual_block_forward or many_tiles or forward' -x -q --timeout 200 --timeout-method thread" \
 "layers|200|python tools/conv_f32_bench.py 3232 10 res16" \
 "bench|200|python bench.py --also_bf16 0" \
 "bench3w|200|SA_WINO16_3W=1 python bench.py --also_bf16 0" \
 "bench1|200|python bench.py --also_bf16 0" \
 "bench3wb|200|SA_WINO16_3W=1 python bench.py --also_bf16 0" \
 "parity3w|400|SA_WINO16_3W=1 python -u -m pytest tests/test_learner_headline_gpu.py -x -q --timeout 300 --timeout-method thread" \
 "prof3w|300|cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && SA_WINO16_3W=1 rocprofv3 --kernel-trace --stats -d gpurun_out/prof26 -o run -- python3 bench.py --also_bf16 0 --steps 20 --warmup 3"
