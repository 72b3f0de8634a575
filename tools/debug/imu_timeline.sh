#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/imu_tl
export CMHAR_BENCH_PEAK_PROBE=0
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/imu_tl -o run -- \
  python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-trace > gpurun_out/imu_tl.log 2>&1 || exit $?
python tools/debug/imu_timeline.py gpurun_out/imu_tl > gpurun_out/imu_timeline.txt 2>&1
find gpurun_out/imu_tl -name "*kernel_trace.csv" -delete
head -60 gpurun_out/imu_timeline.txt
