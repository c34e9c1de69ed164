bash tools/gpu_session.sh \
 "fused|300|python -u -m pytest tests/test_conv_f32_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "bench|200|python bench.py" \
 "benchskip|200|SA_BENCH_SKIP_H2D=1 python bench.py" \
 "layers|200|python tools/conv_f32_bench.py 3232 10 bwd" \
 "bench1|200|python bench.py" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof32 -o run -- python3 bench.py --also_bf16 0 --steps 20 --warmup 3"
