#!/bin/bash
# tile claiming in the persistent GEMM: GEMM tests, GEMM A/B, bench-step A/B and the IMU-branch cost, in-tree vs var/static.so
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "gemm" tests/test_production_shapes_gpu.py > gpurun_out/r06d_tests.log 2>&1 \
  || { tail -30 gpurun_out/r06d_tests.log; exit 1; }
tail -2 gpurun_out/r06d_tests.log
tools/debug/ab_quick.sh r06d crossmodal-imu-video-ood-har_amd/cmhar/libcmhar.so var/static.so || exit $?
timeout -k 10 300 python tools/debug/imu_cost.py > gpurun_out/r06d_imu_cost.log 2>&1 || exit $?
tail -3 gpurun_out/r06d_imu_cost.log
CMHAR_LIB=$PWD/var/static.so timeout -k 10 300 python tools/debug/imu_cost.py > gpurun_out/r06d_imu_cost_static.log 2>&1 || exit $?
tail -3 gpurun_out/r06d_imu_cost_static.log
