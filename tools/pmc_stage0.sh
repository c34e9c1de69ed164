# PMC passes over the fp32 bench's stage-0 kernels (one counter set per run)
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVES"
P2="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"
R="conv_pool_fwd|pool_wgrad|conv_fwd_kernel<16, 16"
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-include-regex "$R" -d gpurun_out/pmcs1 -o run --output-format csv -- python3 bench.py --also_bf16 0 --steps 2 --warmup 1 --graph 0 > gpurun_out/pmcs1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-include-regex "$R" -d gpurun_out/pmcs2 -o run --output-format csv -- python3 bench.py --also_bf16 0 --steps 2 --warmup 1 --graph 0 > gpurun_out/pmcs2.log 2>&1
