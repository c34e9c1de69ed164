P="cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats"
bash tools/gpu_session.sh \
 "bf16|200|python bench.py --dtype bf16" \
 "bf16b|200|python bench.py --dtype bf16" \
 "instr|300|python bench.py --also_bf16 0 --instructions 1" \
 "noinstr|300|python bench.py --also_bf16 0" \
 "profbf|300|$P -d gpurun_out/profbf -o run -- python3 bench.py --dtype bf16 --steps 20 --warmup 3" \
 "prof32|300|$P -d gpurun_out/prof32 -o run -- python3 bench.py --also_bf16 0 --steps 20 --warmup 3"
