C="python experiment.py --level_name=synthetic --torso=deep --unroll_length=8 --synthetic_episode_length=10 --num_actors=4 --batch_size=4 --total_environment_frames=1280 --save_summaries_secs=0"
for v in "fp32 true" "fp32 false" "bf16 true" "bf16 false"; do set -- $v
  timeout -k 10 100 $C --dtype=$1 --trajectory_queue=$2 --logdir=/tmp/e_$1_$2 > gpurun_out/es_$1_$2.log 2>&1; echo "$1 $2 rc=$?" >> gpurun_out/es_summary.txt
done
