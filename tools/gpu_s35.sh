bash tools/gpu_session.sh \
 "gemm|300|python -u -m pytest tests/test_gemm_f32_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "bench|200|python bench.py --also_bf16 0" \
 "benchrm1|200|SA_GEMM_RM=1 python bench.py --also_bf16 0" \
 "bench1|200|python bench.py --also_bf16 0" \
 "parity|500|python -u -m pytest tests/test_learner_parity_gpu.py tests/test_learner_headline_gpu.py -x -q --timeout 300 --timeout-method thread" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof35 -o run -- python3 bench.py --also_bf16 0 --steps 20 --warmup 3"
