bash tools/gpu_session.sh \
 "lstm16|300|SA_LSTM_ROWS=16 python -u -m pytest tests/test_kernels_gpu.py -q -k lstm --timeout 120 --timeout-method thread" \
 "bench32|200|python bench.py --also_bf16 0" \
 "bench16|200|SA_LSTM_ROWS=16 python bench.py --also_bf16 0" \
 "bench32b|200|python bench.py --also_bf16 0" \
 "bench16b|200|SA_LSTM_ROWS=16 python bench.py --also_bf16 0" \
 "tests|300|python -u -m pytest tests/test_learner_parity_gpu.py -q -m gpu --timeout 300 --timeout-method thread"
