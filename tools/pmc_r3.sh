# Round-3 PMC passes over every layer of tools/conv_f32_bench.py (fwd/dgrad/
# wgrad, fused backward, pools): two SQ passes + HBM fetch / write passes.
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_LEVEL_WAVES SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES"
run() {
  timeout -s KILL 120 rocprofv3 --pmc $2 -d gpurun_out/$1 -o run --output-format csv -- python3 tools/conv_f32_bench.py 3232 2 "$3" > gpurun_out/$1.log 2>&1
}
run pmc1 "$P1" "${1:-}" && run pmc2 "$P2" "${1:-}" && run pmc3 "FETCH_SIZE" "${1:-}" && run pmc4 "WRITE_SIZE" "${1:-}"
