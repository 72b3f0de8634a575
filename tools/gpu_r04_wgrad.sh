#!/bin/bash
# Round-4 weight-gradient session: the product build (8-phase transposed-read instantiations issue their LDS-DMA by
# inline asm, so hipcc no longer drains the prefetch before every ds_read_b64_tr_b16) against var/libD0.so
# (-DCMHAR_GEMM8P_ASM_DMA=0, the builtin DMA) in one process; the GEMM parity tests; the step both ways (two builds:
# the product and libD0 copied over it in a scratch tree).
# usage: tools/gpu_r04_wgrad.sh TAG
TAG=${1:-r04w}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
echo "== tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
  -k "bench_gemm or production or gemm or wgrad or transposed or dataparallel or bf16" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_pytest.log; [ $rc -gt 1 ] && exit $rc
echo "== gemm A/B (A = asm DMA, B = builtin DMA)"
timeout -k 10 400 python -u tools/debug/gemm_ab.py crossmodal-imu-video-ood-har_amd/cmhar/libcmhar.so var/libD0.so \
  --epi --rounds 5 > gpurun_out/${TAG}_gemm_ab.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${TAG}_gemm_ab.log
echo "== bench"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_asm.log 2>&1 || exit $?
echo "asm $(tail -1 gpurun_out/${TAG}_bench_asm.log | cut -c1-200)"
exit 0
