#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/wg_fetch gpurun_out/wg_write
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/wg_fetch -o run -- \
  python tools/debug/pmc_wgrad.py run > gpurun_out/wg_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/wg_write -o run -- \
  python tools/debug/pmc_wgrad.py run > gpurun_out/wg_write.log 2>&1 || exit $?
python tools/debug/pmc_wgrad.py report gpurun_out/wg_fetch gpurun_out/wg_write | tee gpurun_out/wg_traffic.txt
