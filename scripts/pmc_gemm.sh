#!/bin/bash
# PMC counter passes for one GEMM shape: scripts/pmc_gemm.sh <tag> <prof_gemm args...>
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_$tag
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc_$tag/p1 -o run -- python3 scripts/prof_gemm.py "$@" > gpurun_out/pmc_$tag/p1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_MFMA --output-format csv -d gpurun_out/pmc_$tag/p2 -o run -- python3 scripts/prof_gemm.py "$@" > gpurun_out/pmc_$tag/p2.log 2>&1
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/pmc_$tag/p3 -o run -- python3 scripts/prof_gemm.py "$@" > gpurun_out/pmc_$tag/p3.log 2>&1
