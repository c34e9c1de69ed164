# Full GPU check of the committed tree: gpu tests, smoke, default bench line,
# fp32 kernel trace (outputs under gpurun_out/)
set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rc_gputest.log 2>&1
echo "gpu tests: $(tail -1 gpurun_out/rc_gputest.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rc_smoke.log 2>&1
echo "smoke ok"
timeout -k 10 300 python bench.py > gpurun_out/rc_bench.log 2>&1
grep '"metric"' gpurun_out/rc_bench.log
timeout -k 10 300 python bench.py --torso shallow --also_bf16 0 > gpurun_out/rc_bench_shallow.log 2>&1
grep '"metric"' gpurun_out/rc_bench_shallow.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rc_prof -o run -- python3 bench.py --also_bf16 0 --steps 20 --warmup 3 > gpurun_out/rc_prof.log 2>&1
