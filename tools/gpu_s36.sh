bash tools/gpu_session.sh \
 "fused|300|python -u -m pytest tests/test_conv_f32_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "test3|300|SA_WINO_CFG=3 python -u -m pytest tests/test_conv_f32_gpu.py -k 'forward or many_tiles or residual_block' -x -q --timeout 200 --timeout-method thread" \
 "layers|200|python tools/conv_f32_bench.py 3232 10 res16" \
 "layers3|200|SA_WINO_CFG=3 python tools/conv_f32_bench.py 3232 10 res16" \
 "bench|200|python bench.py" \
 "bench3|200|SA_WINO_CFG=3 python bench.py --also_bf16 0" \
 "headline|400|python -u -m pytest tests/test_learner_headline_gpu.py tests/test_learner_parity_gpu.py -x -q --timeout 300 --timeout-method thread"
