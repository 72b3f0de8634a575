#!/bin/bash
# A/B of fused-IMU library builds (CMHAR_LIB): IMU branch wall time + rocprofv3 kernel summary each, plus the IMU
# parity tests on the product build.  usage: tools/debug/imu_kc_ab.sh TAG lib1.so lib2.so ...
TAG=$1; shift
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_imu_fused_gpu.py tests/test_models_gpu.py tests/test_trainers_gpu.py \
  -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 \
  || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for lib in "$@"; do
  n=$(basename $lib .so)
  CMHAR_LIB=$PWD/$lib timeout -k 10 300 python tools/debug/imu_bench.py > gpurun_out/${TAG}_${n}.log 2>&1 || exit $?
  echo "$n: $(tail -1 gpurun_out/${TAG}_${n}.log)"
  rm -rf gpurun_out/${TAG}_${n}_prof
  CMHAR_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_${n}_prof -o run -- \
    python tools/debug/imu_bench.py > gpurun_out/${TAG}_${n}_prof.log 2>&1 || exit $?
  python tools/rocpd_summary.py $(find gpurun_out/${TAG}_${n}_prof -name "*.db" | head -1) 2>/dev/null | grep -E "imu_encoder|TOTAL"
done
exit 0
