#!/bin/bash
# GEMM per-shape A/B (tools/debug/gemm_ab.py --epi) + bench-step A/B over library builds.  usage: ab_quick.sh TAG lib...
TAG=$1; shift
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/debug/gemm_ab.py "$@" --epi --rounds 5 > gpurun_out/${TAG}_gemm_ab.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_gemm_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_gemm_ab.log
tools/debug/lib_step_ab.sh ${TAG}_step "$@"
