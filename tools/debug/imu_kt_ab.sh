#!/bin/bash
# A/B of the few-tile fp32 GEMM K-tile inside the bench step: per library build, a rocprofv3 kernel trace of a short
# bench run (IMU GEMM kernel-ms under contention) and tools/debug/imu_cost.py (wall cost of the IMU branch).
# usage: tools/debug/imu_kt_ab.sh lib1.so lib2.so ...   (outputs gpurun_out/ktab_<name>*)
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in "$@"; do
  n=$(basename $lib .so)
  rm -rf gpurun_out/ktab_$n
  CMHAR_LIB=$(realpath $lib) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ktab_$n -o run -- \
    python bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/ktab_$n.log 2>&1 || exit $?
  find gpurun_out/ktab_$n -name "*kernel_trace.csv" -delete
  CMHAR_LIB=$(realpath $lib) timeout -k 10 300 python tools/debug/imu_cost.py > gpurun_out/ktab_${n}_cost.log 2>&1 || exit $?
done
