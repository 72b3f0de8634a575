#!/bin/bash
# Round-4 triple-buffered-A session: the product build (8-phase forward/dgrad layouts with three A buffers) against
# var/libN2.so (-DCMHAR_GEMM8P_NA_DEFAULT=2) and var/libW3.so (weight-gradient layout with three A buffers too), in
# one process on the step's GEMM shapes; the GEMM parity tests; the step alternated with CMHAR_GEMM8P_NA=3 / 2.
# usage: tools/gpu_r04_na.sh TAG
TAG=${1:-r04n}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
echo "== tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
  -k "bench_gemm or production or gemm or wgrad or transposed" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_pytest.log; [ $rc -gt 1 ] && exit $rc
echo "== gemm A/B (A = fwd NA3 / wgrad NA2, B = fwd NA2, C = fwd NA3 / wgrad NA3)"
timeout -k 10 400 python -u tools/debug/gemm_ab.py crossmodal-imu-video-ood-har_amd/cmhar/libcmhar.so var/libN2.so var/libW3.so \
  --epi --rounds 5 > gpurun_out/${TAG}_gemm_ab.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${TAG}_gemm_ab.log
echo "== bench"
for v in 3 2 3 2; do
  CMHAR_GEMM8P_NA=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_$v.log 2>&1 || exit $?
  echo "na=$v $(tail -1 gpurun_out/${TAG}_bench_$v.log | cut -c1-200)"
done
exit 0
