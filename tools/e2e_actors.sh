#!/bin/bash
# End-to-end actor -> learner throughput on one GPU (synthetic DMLab-shaped
# env, deep torso, B=32, T=100): actor threads in the learner process vs
# vectorised actor-group processes.  usage: tools/e2e_actors.sh TAG ACTORS GROUPS [extra flags]
tag=$1; actors=$2; groups=$3; shift 3
mkdir -p gpurun_out
timeout -k 10 240 python experiment.py --level_name=synthetic --torso=deep \
  --num_actors=$actors --actor_groups=$groups --batch_size=32 --unroll_length=100 \
  --total_environment_frames=${FRAMES:-3072000} --log_every_frames=256000 \
  --save_summaries_secs=10 --save_checkpoint_secs=100000 \
  --logdir=/tmp/e2e_$tag "$@" > gpurun_out/e2e_$tag.log 2>&1
rc=$?
grep -E "frames/s|actor group|Error|error" gpurun_out/e2e_$tag.log | grep -v "Episode return" | tail -8
exit $rc
