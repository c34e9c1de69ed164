bash tools/gpu_session.sh \
 "gputests|1000|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench|200|python bench.py"
