bash tools/gpu_session.sh \
 "wcheck|180|python tools/wino_check.py 37" \
 "cbench|200|python tools/conv_f32_bench.py 3232 5 deep; python tools/conv_f32_bench.py 3232 5 bwd" \
 "bench|300|python bench.py --also_bf16 0" \
 "tests|500|python -u -m pytest tests/test_learner_parity_gpu.py -q -m gpu --timeout 300 --timeout-method thread"
