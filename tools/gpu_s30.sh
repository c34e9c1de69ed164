bash tools/gpu_session.sh \
 "bf16only|200|python bench.py --dtype bf16" \
 "proffull|300|cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof30 -o run -- python3 bench.py --steps 20 --warmup 3" \
 "profbf16|300|cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof30b -o run -- python3 bench.py --dtype bf16 --also_bf16 0 --steps 20 --warmup 3"
