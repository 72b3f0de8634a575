#!/bin/bash
# Round-5 session: attention A/B of library variants (in one process) + PMC traffic of the QKV forward GEMM alone.
# usage: tools/gpu_r05_attn.sh TAG libA.so libB.so [...]
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
echo "== attn A/B"
timeout -k 10 300 python tools/debug/attn_ab.py "$@" --prescaled --rounds 9 > gpurun_out/${TAG}_attn_ab.log 2>&1 || exit $?
cat gpurun_out/${TAG}_attn_ab.log
if [ -n "$GEMM_PMC" ]; then
  echo "== qkv fwd traffic"
  for P in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum"; do
    n=$(echo $P | cut -c1-5)
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/${TAG}_qkv_$n -o run -- \
      python tools/debug/gemm_one.py qkv fwd 5 > gpurun_out/${TAG}_qkv_$n.log 2>&1 || exit $?
    python tools/pmc_summary.py gpurun_out/${TAG}_qkv_$n gemm > gpurun_out/${TAG}_qkv_$n.txt 2>&1
    cat gpurun_out/${TAG}_qkv_$n.txt | head -8
    find gpurun_out/${TAG}_qkv_$n -name "*.csv" -size +5M -delete
  done
fi
exit 0
