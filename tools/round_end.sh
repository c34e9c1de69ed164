#!/bin/bash
# Round-end evidence on one GPU box: GPU tests, smoke, every bench line of
# profiles/rN_bench_1gpu.jsonl, kernel traces of the fp32 and bf16 steps
# (rocpd db: tools/prof_summary.py, tools/timeline.py).  Outputs under
# gpurun_out/re/.  Each GPU step has its own limit; the first failure ends it.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/re
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
echo "gpu tests: $(tail -1 $O/gputest.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > $O/b_$n.log 2>&1
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $O/b_$n.log | head -1)"
}
run default
run atari_bf16 --dtype bf16 --height 84 --width 84 --channels 4
run atari_fp32 --height 84 --width 84 --channels 4 --also_bf16 0
run popart --popart 30 --also_bf16 0
run instr --instructions 1 --also_bf16 0
run shallow --torso shallow --also_bf16 0
run doom --height 72 --width 128
SA_DIST_BACKEND=gloo run dp2_gloo --gpus 2 --also_bf16 0 --steps 10
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pf32 -o run -- python3 bench.py --also_bf16 0 --steps 20 --warmup 3 > $O/pf32.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pbf16 -o run -- python3 bench.py --dtype bf16 --steps 20 --warmup 3 > $O/pbf16.log 2>&1
echo done
