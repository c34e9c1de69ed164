bash tools/gpu_session.sh \
 "fused|300|python -u -m pytest tests/test_conv_f32_gpu.py -k 'bwd_fused' -x -q --timeout 200 --timeout-method thread" \
 "fusedv2|300|SA_FUSED16_V2=1 python -u -m pytest tests/test_conv_f32_gpu.py -k 'bwd_fused' -x -q --timeout 200 --timeout-method thread" \
 "layers|200|python tools/conv_f32_bench.py 3232 10 bwd" \
 "layersv2|200|SA_FUSED16_V2=1 python tools/conv_f32_bench.py 3232 10 bwd" \
 "bench|200|python bench.py --also_bf16 0" \
 "benchv2|200|SA_FUSED16_V2=1 python bench.py --also_bf16 0" \
 "bench1|200|python bench.py --also_bf16 0" \
 "benchv2b|200|SA_FUSED16_V2=1 python bench.py --also_bf16 0"
bash tools/gpu_session.sh \
 "ablate2|200|SA_WINO_ABLATE=2 python tools/conv_f32_bench.py 3232 10 res" \
 "pmc|300|bash tools/pmc_fused.sh"
