#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (tools/debug/pmc_calib.py)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/calib_fetch gpurun_out/calib_write
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib_fetch -o run -- \
  python tools/debug/pmc_calib.py > gpurun_out/calib_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib_write -o run -- \
  python tools/debug/pmc_calib.py > gpurun_out/calib_write.log 2>&1 || exit $?
python tools/pmc_traffic.py gpurun_out/calib_fetch gpurun_out/calib_write gpurun_out/calib_traffic.json calib calib \
  > gpurun_out/calib_traffic.txt 2>&1 || exit $?
cat gpurun_out/calib_traffic.txt
