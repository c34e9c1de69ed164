bash tools/gpu_session.sh \
 "tests|400|python -u -m pytest tests/test_conv_f32_gpu.py tests/test_learner_parity_gpu.py tests/test_learner_headline_gpu.py -q -x --timeout 300 --timeout-method thread" \
 "layers|200|python tools/conv_f32_bench.py 3232 10 res16" \
 "layers0|200|SA_FUSED_BWD_WWG=0 python tools/conv_f32_bench.py 3232 10 res16" \
 "bench|200|python bench.py --also_bf16 0" \
 "bench0|200|SA_FUSED_BWD_WWG=0 python bench.py --also_bf16 0" \
 "benchb|200|python bench.py --also_bf16 0"
