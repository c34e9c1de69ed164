#!/bin/bash
# Kernel trace of an end-to-end config-#4 run with the inference board, then
# tools/micro/board_trace.py on the learner process's database; only the
# summary stays under gpurun_out (the database is larger than gpurun's pull
# limit).  Extra experiment.py flags follow.  usage: board_trace.sh TAG [flags]
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag=$1; shift
export TMPDIR=/tmp
D=/tmp/bt_$tag
rm -rf $D
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $D -o run -- \
  python3 experiment.py --level_name=synthetic --torso=deep --batch_size=32 \
  --unroll_length=100 --total_environment_frames=1536000 \
  --log_every_frames=256000 --save_summaries_secs=10 \
  --save_checkpoint_secs=100000 --num_actors=150 --logdir=/tmp/e2e_bt_$tag \
  --popart=true "$@" > gpurun_out/board_trace_$tag.log 2>&1
db=$(python3 -c "import glob,os,sys; f=sorted(glob.glob('$D/**/*.db', recursive=True), key=os.path.getsize); print(f[-1] if f else '')")
python3 tools/micro/board_trace.py "$db" gpurun_out/board_trace_$tag.txt
rm -rf $D
