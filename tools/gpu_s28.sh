bash tools/gpu_session.sh \
 "gemm|300|python -u -m pytest tests/test_gemm_f32_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "bench|200|python bench.py --also_bf16 0" \
 "bench1|200|python bench.py --also_bf16 0" \
 "gputests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof28 -o run -- python3 bench.py --also_bf16 0 --steps 20 --warmup 3"
