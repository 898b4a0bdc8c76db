#!/bin/bash
# SQ issue/wait counters of the cn_linear variants of one operand mode (GEMM_MODE).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
M6=${GEMM_MODE:-x6}
export GEMM_MODE=$M6
mkdir -p $R/gpurun_out/sq
timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/sq/p1_$M6 -o p1 --output-format csv -- python3 $R/tools/gemm_prof.py
timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MFMA_F SQ_INSTS_LDS SQ_INSTS_SALU -d $R/gpurun_out/sq/p2_$M6 -o p2 --output-format csv -- python3 $R/tools/gemm_prof.py
timeout -k 10 180 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT -d $R/gpurun_out/sq/p3_$M6 -o p3 --output-format csv -- python3 $R/tools/gemm_prof.py
