bash tools/gpu_session.sh \
 "tests|300|python -u -m pytest tests/test_board_native_gpu.py -x -v --timeout 120 --timeout-method thread" \
 "bn96|280|bash tools/e2e_actors.sh bn96 96 2 --inference_server=true" \
 "bp96|280|SA_BOARD_NATIVE=0 bash tools/e2e_actors.sh bp96 96 2 --inference_server=true" \
 "g96|280|bash tools/e2e_actors.sh g96 96 1" \
 "bn192|280|bash tools/e2e_actors.sh bn192 192 4 --inference_server=true"
