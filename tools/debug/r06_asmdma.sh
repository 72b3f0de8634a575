#!/bin/bash
# attention LDS-DMA by inline asm: kernel A/B (previous HEAD, in-tree = builtin DMA + retired fragments, asm DMA) and
# the bench step alternated over the three builds
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/debug/attn_ab.py var/prev.so crossmodal-imu-video-ood-har_amd/cmhar/libcmhar.so \
  var/asmdma.so --prescaled --rounds 7 > gpurun_out/r06r_attn_ab.log 2>&1 || { tail -20 gpurun_out/r06r_attn_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06r_attn_ab.log
tools/debug/lib_step_ab.sh r06r_step var/prev.so var/asmdma.so
