#!/bin/bash
# Three rocprofv3 --pmc passes (issue / MFMA / LDS counters) over one command; each pass its own run.
#   tools/debug/pmc_run.sh NAME python tools/debug/f32_gemm_bench.py ...
# then: python tools/pmc_summary.py gpurun_out/pmc_NAME<i> [kernel-substring]
export TMPDIR=/tmp
NAME=$1; shift
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F SQ_ACTIVE_INST_LDS"
P3="SQ_INSTS_VMEM_RD SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_WAVES SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_$NAME$i -o run -- "$@" > gpurun_out/pmc_$NAME$i.log 2>&1 || exit $?
done
echo done
