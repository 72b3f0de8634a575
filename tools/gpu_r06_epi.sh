#!/bin/bash
# Round 6: register-direct GEMM epilogue (CMHAR_EPI_DIRECT).  GEMM parity tests on the in-tree build, then the
# per-shape A/B (tools/debug/gemm_ab.py --epi) and the bench step alternated over the given library builds.
# usage: tools/gpu_r06_epi.sh TAG lib.so...   (the in-tree library is always the first arm)
TAG=$1; shift
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "gemm or wgrad or tubelet or dgrad or attn or attention" tests/test_production_shapes_gpu.py \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
LIBS="crossmodal-imu-video-ood-har_amd/cmhar/libcmhar.so $*"
timeout -k 10 400 python -u tools/debug/gemm_ab.py $LIBS --epi --rounds 5 > gpurun_out/${TAG}_gemm_ab.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_gemm_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_gemm_ab.log
tools/debug/lib_step_ab.sh ${TAG}_step $LIBS
