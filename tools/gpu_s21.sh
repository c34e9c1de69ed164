bash tools/gpu_session.sh \
 "a0|100|python tools/conv_f32_bench.py 3232 5 head" \
 "a1|100|SA_FUSED_ABLATE=1 python tools/conv_f32_bench.py 3232 5 head" \
 "a2|100|SA_FUSED_ABLATE=2 python tools/conv_f32_bench.py 3232 5 head" \
 "a4|100|SA_FUSED_ABLATE=4 python tools/conv_f32_bench.py 3232 5 head" \
 "a6|100|SA_FUSED_ABLATE=6 python tools/conv_f32_bench.py 3232 5 head"
