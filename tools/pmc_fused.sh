# PMC passes over the fused conv backward kernels (tools/conv_f32_bench.py 'bwd' rows)
# and the Winograd forward kernels ('deep' layer rows); one counter group per pass
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVES"
P2="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"
timeout -s KILL 90 rocprofv3 --pmc $P1 -d gpurun_out/pmcf1 -o run --output-format csv -- python3 tools/conv_f32_bench.py 3232 2 deep > gpurun_out/pmcf1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc $P2 -d gpurun_out/pmcf2 -o run --output-format csv -- python3 tools/conv_f32_bench.py 3232 2 deep > gpurun_out/pmcf2.log 2>&1
