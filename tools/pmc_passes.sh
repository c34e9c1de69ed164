#!/bin/bash
# Two SQ counter passes (one counter group per rocprofv3 run, each under its
# own time limit) over any command; read the CSVs with tools/pmc_table.py.
# usage: tools/pmc_passes.sh <out-name> <command...>
#   e.g. tools/pmc_passes.sh pmcf python3 tools/conv_f32_bench.py 3232 2 deep
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
name=$1; shift
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVES"
P2="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"
P3="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE"
i=1
for P in "$P1" "$P2" ${PMC_FETCH:+"$P3"}; do
  timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/${name}$i -o run \
      --output-format csv -- "$@" > gpurun_out/${name}$i.log 2>&1
  i=$((i + 1))
done
