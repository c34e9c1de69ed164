bash tools/gpu_session.sh \
 "bench|200|python bench.py" \
 "benchskip|200|SA_BENCH_SKIP_H2D=1 python bench.py"
