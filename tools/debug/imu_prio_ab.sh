#!/bin/bash
# What the IMU branch costs the bench step (tools/debug/imu_cost.py: side stream / main stream / stub) with the side
# stream at default and at high priority.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in 0 -1 0 -1; do
  CMHAR_IMU_STREAM_PRIORITY=$p timeout -k 10 300 python tools/debug/imu_cost.py > gpurun_out/imuprio_$p.log 2>&1 || exit $?
  echo "priority $p:"; grep -E "stream|stub" gpurun_out/imuprio_$p.log
done
exit 0
