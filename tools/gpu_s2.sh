bash tools/gpu_session.sh \
 "wcheck|120|python tools/wino_check.py 37" \
 "tests|600|python -u -m pytest tests/test_gemm_f32_gpu.py tests/test_learner_parity_gpu.py tests/test_conv_f32_gpu.py tests/test_lang_lstm_gpu.py tests/test_learner_headline_gpu.py tests/test_train_dp.py -q -m gpu --timeout 300 --timeout-method thread" \
 "bench|300|python bench.py --also_bf16 1" \
 "benchi|300|python bench.py --also_bf16 1 --instructions 1" \
 "cfg|200|bash tools/exp_wino_cfg.sh"
