bash tools/gpu_session.sh \
 "learner|600|python -u -m pytest tests/test_learner_gpu.py tests/test_dp_gpu.py -x -q --timeout 300 --timeout-method thread" \
 "lstmw8|300|SA_LSTM_BWD_W8=1 python -u -m pytest tests/test_kernels_gpu.py tests/test_learner_headline_gpu.py -x -q -k 'lstm or headline' --timeout 300 --timeout-method thread" \
 "bench|200|python bench.py" \
 "benchw8|200|SA_LSTM_BWD_W8=1 python bench.py --also_bf16 0" \
 "bench1|200|python bench.py" \
 "benchw8b|200|SA_LSTM_BWD_W8=1 python bench.py --also_bf16 0"
