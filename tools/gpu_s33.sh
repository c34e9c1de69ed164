bash tools/gpu_session.sh \
 "gputests|1000|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench|200|python bench.py" \
 "bench1|200|python bench.py" \
 "layers|200|python tools/conv_f32_bench.py 3232 10 bwd" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof33 -o run -- python3 bench.py --also_bf16 0 --steps 20 --warmup 3"
