#!/bin/bash
# Round-5 measurement session: torch.matmul (hipBLASLt) vs the library on every VideoMAE GEMM shape, then a
# rocprofv3 kernel trace of the bench step (per-kernel table + idle-interval attribution).
# usage: tools/gpu_r05_prof.sh TAG
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
echo "== gemm vs hipBLASLt"
timeout -k 10 300 python tools/debug/gemm_ab.py crossmodal-imu-video-ood-har_amd/cmhar/libcmhar.so --torch --rounds 5 \
  > gpurun_out/${TAG}_gemm_torch.log 2>&1 || exit $?
cat gpurun_out/${TAG}_gemm_torch.log
echo "== kernel trace"
bash tools/prof_step.sh ${TAG} || exit $?
cat gpurun_out/${TAG}_kernels.txt | tail -22
exit 0
