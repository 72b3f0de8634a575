#!/bin/bash
# The fused IMU encoder forward: bit-identity / parity tests, then the IMU branch (tools/debug/imu_bench.py, B = 32,
# 6x200, fwd+bwd) with the fused forward (CMHAR_IMU_FUSED=1) and the per-op launches (=0), wall time and
# rocprofv3 kernel summaries.  usage: tools/debug/imu_fused_ab.sh TAG
TAG=${1:-imuf}
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_imu_fused_gpu.py tests/test_models_gpu.py tests/test_trainers_gpu.py \
  tests/test_geometries_gpu.py -x -q -p no:cacheprovider --timeout 180 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
for v in 1 0; do
  CMHAR_IMU_FUSED=$v timeout -k 10 300 python tools/debug/imu_bench.py > gpurun_out/${TAG}_bench$v.log 2>&1 || exit $?
  echo "fused=$v: $(tail -1 gpurun_out/${TAG}_bench$v.log)"
  rm -rf gpurun_out/${TAG}_prof$v
  CMHAR_IMU_FUSED=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof$v -o run -- \
    python tools/debug/imu_bench.py > gpurun_out/${TAG}_prof$v.log 2>&1 || exit $?
  find gpurun_out/${TAG}_prof$v -name "*kernel_trace.csv" -delete
done
exit 0
