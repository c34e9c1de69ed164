#!/bin/bash
# A/B sweep of one environment knob over the fp32 bench (or any command that
# prints the bench JSON line): one run per value, each under its own limit,
# stopping at the first failure.
# usage: tools/ab_env.sh VAR "v1 v2 ..." [command...]
#   default command: python bench.py --also_bf16 0 --steps 20 --warmup 5
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
var=$1; vals=$2; shift 2
[ $# -gt 0 ] || set -- python bench.py --also_bf16 0 --steps 20 --warmup 5
for v in $vals; do
  env "$var=$v" timeout -k 10 200 "$@" > "gpurun_out/ab_${var}_$v.log" 2>&1
  echo "$var=$v $(grep -o '"ms_per_step": [0-9.]*' "gpurun_out/ab_${var}_$v.log" | head -1)"
done
