#!/bin/bash
# optimistic attention forward: the new tests + the attention / production-shape / fp16 suites, the kernel A/B
# against the exact single launch (previous build) and the bench step alternated with it
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_attention_fwd_opt_gpu.py \
  tests/test_production_shapes_gpu.py -k "attention or flash or optimistic" > gpurun_out/r06o_tests.log 2>&1 || { tail -30 gpurun_out/r06o_tests.log; exit 1; }
tail -3 gpurun_out/r06o_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp16_gpu.py \
  tests/test_fusion_gpu.py > gpurun_out/r06o_tests2.log 2>&1 || { tail -30 gpurun_out/r06o_tests2.log; exit 1; }
tail -2 gpurun_out/r06o_tests2.log
timeout -k 10 300 python -u tools/debug/attn_ab.py var/base.so crossmodal-imu-video-ood-har_amd/cmhar/libcmhar.so --prescaled --rounds 9 \
  > gpurun_out/r06o_attn_ab.log 2>&1 || { tail -20 gpurun_out/r06o_attn_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06o_attn_ab.log
for rep in 1 2; do
  for opt in 0 1; do
    CMHAR_ATTN_FWD_OPT=$opt timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline \
      > gpurun_out/r06o_step_${opt}_${rep}.log 2>&1 || exit $?
    echo "fwd_opt=$opt rep=$rep $(tail -1 gpurun_out/r06o_step_${opt}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]; print(d["value"], d["ms_per_step"], k["attn_fwd_bf16"])')"
  done
done
