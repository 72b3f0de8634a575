#!/bin/bash
# PMC passes over the R3D-18 implicit-GEMM conv kernels (tools/debug/conv_bench.py, one layer set), each pass with
# GRBM_GUI_ACTIVE for per-cycle normalisation; summary by tools/debug/pmc_table.py.
# usage: tools/debug/pmc_conv.sh TAG LAYERS   (LAYERS: conv_bench --layers, e.g. layer1)
TAG=$1; LAYERS=$2
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE"
P3="SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
i=0
dirs=""
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  rm -rf gpurun_out/${TAG}_pmc$i
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/${TAG}_pmc$i -o run -- \
    python tools/debug/conv_bench.py --layers $LAYERS --reps 2 > gpurun_out/${TAG}_pmc$i.log 2>&1 || exit $?
  dirs="$dirs gpurun_out/${TAG}_pmc$i"
done
python tools/debug/pmc_table.py conv3d_ $dirs > gpurun_out/${TAG}_pmc_conv.txt 2>&1 || exit $?
find $dirs -name "*.csv" -size +20M -delete
echo done
