bash tools/gpu_session.sh \
 "layers|300|python tools/conv_f32_bench.py 3232 10" \
 "benchfull|300|python bench.py" \
 "shallow|200|python bench.py --torso shallow --also_bf16 0" \
 "instr|200|python bench.py --instructions 1 --also_bf16 0" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof29 -o run -- python3 bench.py --also_bf16 0 --steps 20 --warmup 3"
