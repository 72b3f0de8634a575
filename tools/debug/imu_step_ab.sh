#!/bin/bash
# The bench step (B = 32, 16x224^2 + IMU 6x200) with the fused IMU encoder (CMHAR_IMU_FUSED=1) and the per-op
# launches (=0), alternated twice; then the IMU parity tests.  usage: tools/debug/imu_step_ab.sh TAG
TAG=${1:-imustep}
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_imu_fused_gpu.py tests/test_models_gpu.py tests/test_trainers_gpu.py \
  tests/test_geometries_gpu.py -x -q -p no:cacheprovider --timeout 180 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for rep in 1 2; do
  for v in 1 0; do
    CMHAR_IMU_FUSED=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-trace \
      > gpurun_out/${TAG}_b${v}_${rep}.log 2>&1 || exit $?
    echo "fused=$v rep=$rep $(tail -1 gpurun_out/${TAG}_b${v}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
exit 0
