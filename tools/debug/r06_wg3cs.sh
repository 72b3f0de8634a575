#!/bin/bash
# nine-tap weight gradient with 32 channels per workgroup (two workgroups per CU) vs 64: R3D tests under
# CMHAR_WGRAD3_CS=32, per-layer conv timing and the R3D-18 bench alternated under both values
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
CMHAR_WGRAD3_CS=32 timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu \
  tests/test_r3d_gpu.py tests/test_r3d_production_gpu.py > gpurun_out/r06w_tests.log 2>&1 \
  || { tail -30 gpurun_out/r06w_tests.log; exit 1; }
tail -2 gpurun_out/r06w_tests.log
for cs in 64 32; do
  CMHAR_WGRAD3_CS=$cs timeout -k 10 300 python tools/debug/conv_bench.py > gpurun_out/r06w_conv_$cs.log 2>&1 || exit $?
  echo "== conv_bench CS=$cs"; grep -v amdgpu.ids gpurun_out/r06w_conv_$cs.log
done
for rep in 1 2; do
  for cs in 64 32; do
    CMHAR_WGRAD3_CS=$cs timeout -k 10 300 python tools/bench_r3d.py > gpurun_out/r06w_r3d_${cs}_$rep.log 2>&1 || exit $?
    echo "r3d CS=$cs rep=$rep $(tail -1 gpurun_out/r06w_r3d_${cs}_$rep.log | cut -c1-200)"
  done
done
