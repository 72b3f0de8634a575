#!/bin/bash
# Round-5 session: GEMM A/B of library variants on every VideoMAE-B GEMM shape (one process), the QKV forward's PMC
# traffic per variant, then the bench step alternated over the variants.
# usage: tools/gpu_r05_gemm.sh TAG libA.so libB.so [...]
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
echo "== gemm A/B"
timeout -k 10 400 python tools/debug/gemm_ab.py "$@" --epi --rounds 7 > gpurun_out/${TAG}_gemm_ab.log 2>&1 || exit $?
cat gpurun_out/${TAG}_gemm_ab.log
echo "== qkv / fc1 fwd traffic per variant"
for lib in "$@"; do
  n=$(basename $lib .so)
  for shape in qkv fc1; do
    CMHAR_LIB=$PWD/$lib timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_${n}_${shape} -o run -- \
      python tools/debug/gemm_one.py $shape fwd 5 > gpurun_out/${TAG}_${n}_${shape}.log 2>&1 || exit $?
    echo "$n $shape $(python tools/pmc_summary.py gpurun_out/${TAG}_${n}_${shape} gemm | grep FETCH_SIZE)"
    find gpurun_out/${TAG}_${n}_${shape} -name "*.csv" -size +5M -delete
  done
done
if [ -n "$STEP_AB" ]; then
  echo "== step A/B"
  bash tools/debug/lib_step_ab.sh ${TAG}_step "$@" || exit $?
fi
exit 0
