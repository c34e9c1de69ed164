export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_LEVEL_WAVES SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES"
timeout -s KILL 90 rocprofv3 --pmc $P1 -d gpurun_out/pmc1 -o run --output-format csv -- python tools/conv_f32_bench.py 3232 2 deep > gpurun_out/pmc1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc $P2 -d gpurun_out/pmc2 -o run --output-format csv -- python tools/conv_f32_bench.py 3232 2 deep > gpurun_out/pmc2.log 2>&1
