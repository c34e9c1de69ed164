bash tools/gpu_session.sh \
 "fusedtest|300|python -u -m pytest tests/test_conv_f32_gpu.py -k 'bwd_fused or many_tiles' -x -q --timeout 200 --timeout-method thread" \
 "layers|200|python tools/conv_f32_bench.py 3232 10 res32" \
 "bench|200|python bench.py --also_bf16 0" \
 "bench0|200|SA_FUSED_BWD32=0 python bench.py --also_bf16 0" \
 "gputests|900|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof19 -o run -- python3 bench.py --also_bf16 0 --steps 20 --warmup 3"
