bash tools/gpu_session.sh \
 "fused|300|python -u -m pytest tests/test_conv_f32_gpu.py -k 'bwd_fused' -x -q --timeout 200 --timeout-method thread" \
 "layers|200|python tools/conv_f32_bench.py 3232 10 bwd" \
 "bench|200|python bench.py --also_bf16 0" \
 "bench1|200|python bench.py --also_bf16 0" \
 "pmc|300|bash tools/pmc_fused.sh"
