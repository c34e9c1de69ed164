#!/bin/bash
# End-to-end actor -> learner throughput at the BASELINE actor configs on one
# GPU box, each run under the host CPU sampler (tools/micro/cpu_sampler.py):
#   cfg2: 48 actors, Atari-shaped 84x84x4 synthetic frames, bf16 learner
#   cfg4: 150 actors, PopArt value normalisation, fp32 learner
# Extra flags for both runs follow the tag (e.g. --envs_per_worker=8);
# E2E_CFGS picks the configs (default "cfg2 cfg4").
# usage: tools/r6_e2e.sh TAG [extra flags]; logs under gpurun_out/e2e/.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
O=gpurun_out/e2e
mkdir -p $O
common="--level_name=synthetic --torso=deep --batch_size=32 --unroll_length=100 \
  --total_environment_frames=${FRAMES:-4096000} --log_every_frames=256000 \
  --save_summaries_secs=10 --save_checkpoint_secs=100000"
run() {  # name, actors, flags...
  local n=$1 a=$2; shift 2
  timeout -k 10 ${E2E_LIMIT:-240} python tools/micro/cpu_sampler.py $O/${n}_${tag}_cpu.txt -- \
    python experiment.py $common --num_actors=$a --logdir=/tmp/e2e_${n}_${tag} "$@" \
    > $O/${n}_${tag}.log 2>&1
  grep -E "frames/s|inference board" $O/${n}_${tag}.log | tail -4
  tail -6 $O/${n}_${tag}.log | grep -E "role|learner|group|env|total" || true
}
for c in ${E2E_CFGS:-cfg2 cfg4}; do
  case $c in
    cfg2) run cfg2 48 --dtype=bf16 --obs_shape=84x84x4 "$@" ;;
    cfg4) run cfg4 150 --popart=true "$@" ;;
  esac
done
