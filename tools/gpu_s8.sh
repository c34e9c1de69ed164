bash tools/gpu_session.sh \
 "tests|500|python -u -m pytest tests/test_conv_f32_gpu.py tests/test_learner_parity_gpu.py -q -m gpu --timeout 300 --timeout-method thread && SA_F32_U8_DEEP=1 SA_F32_U8_SHALLOW=0 python -u -m pytest tests/test_conv_f32_gpu.py tests/test_learner_parity_gpu.py -q -m gpu --timeout 300 --timeout-method thread -k 'torso or learner'" \
 "bench|200|python bench.py --also_bf16 0" \
 "benchs|200|python bench.py --also_bf16 0 --torso shallow" \
 "benchs0|200|SA_F32_U8_SHALLOW=0 python bench.py --also_bf16 0 --torso shallow" \
 "benchs1|200|python bench.py --also_bf16 0 --torso shallow" \
 "benchs2|200|SA_F32_U8_SHALLOW=0 python bench.py --also_bf16 0 --torso shallow"
