#!/bin/bash
# SQ issue/wait counters for the cn_linear epilogue variants (separate passes).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/sq
rocprofv3 -L > $R/gpurun_out/sq/counters.txt 2>&1 || true
V=${COPENERF_LINEAR_VARIANT:-0}
export COPENERF_LINEAR_VARIANT=$V
timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/sq/p1_v$V -o p1 --output-format csv -- python3 $R/tools/gemm_prof.py
timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MFMA_F SQ_INSTS_LDS SQ_INSTS_SALU -d $R/gpurun_out/sq/p2_v$V -o p2 --output-format csv -- python3 $R/tools/gemm_prof.py
