#!/bin/bash
# Round-4 asm-DMA session: flash kernels with inline-asm LDS-DMA (product) vs var/libA0.so (-DCMHAR_ATTN_DMA_ASM=0);
# the weight-gradient GEMMs with three A buffers (var/libW3.so) vs two (product), both on the asm-DMA 8-phase kernel;
# attention / model / GEMM tests; the step.
# usage: tools/gpu_r04_asmdma.sh TAG
TAG=${1:-r04d}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
echo "== tests"
timeout -k 10 700 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
  -k "attention or flash or videomae or token0 or fusion or bench_gemm or production or wgrad or bf16" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_pytest.log; [ $rc -gt 1 ] && exit $rc
echo "== attention A/B (A = asm DMA, B = builtin DMA)"
timeout -k 10 300 python -u tools/debug/attn_ab.py crossmodal-imu-video-ood-har_amd/cmhar/libcmhar.so var/libA0.so --prescaled \
  > gpurun_out/${TAG}_attn_ab.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${TAG}_attn_ab.log
echo "== gemm A/B (A = wgrad NA2, B = wgrad NA3)"
timeout -k 10 400 python -u tools/debug/gemm_ab.py crossmodal-imu-video-ood-har_amd/cmhar/libcmhar.so var/libW3.so \
  --epi --rounds 5 > gpurun_out/${TAG}_gemm_ab.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${TAG}_gemm_ab.log
echo "== bench"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
echo "$(tail -1 gpurun_out/${TAG}_bench.log | cut -c1-200)"
exit 0
