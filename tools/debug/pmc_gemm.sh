#!/bin/bash
# Counter passes over one GEMM shape: issue/MFMA, LDS, memory hierarchy.  tools/debug/pmc_gemm.sh TAG NAME LAYOUT
export TMPDIR=/tmp
TAG=$1; NAME=$2; LAY=$3
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum"
P4="TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_${TAG}$i -o run -- python tools/debug/gemm_one.py $NAME $LAY 5 > gpurun_out/pmc_${TAG}$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_${TAG}$i.log; }
  python tools/pmc_summary.py gpurun_out/pmc_${TAG}$i gemm > gpurun_out/pmc_${TAG}$i.txt 2>&1
  find gpurun_out/pmc_${TAG}$i -name "*.csv" -size +5M -delete
done
timeout -k 5 60 python tools/debug/gemm_one.py $NAME $LAY 20
echo done
