#!/bin/bash
# Round-4 persistent-GEMM session: A/B of the product build (persistent 8-phase kernel) against var/libB.so (built with
# -DCMHAR_GEMM_PERSIST_DEFAULT=0) on the step's GEMM shapes in one process, the GEMM parity tests, a short bench.
# usage: tools/gpu_r04_persist.sh TAG
TAG=${1:-r04g}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
echo "== tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
  -k "persistent or bench_gemm or production or gemm" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_pytest.log; [ $rc -gt 1 ] && exit $rc
echo "== gemm A/B (A = persistent, B = one tile per workgroup)"
timeout -k 10 300 python -u tools/debug/gemm_ab.py crossmodal-imu-video-ood-har_amd/cmhar/libcmhar.so var/libB.so --epi --rounds 5 \
  > gpurun_out/${TAG}_gemm_ab.log 2>&1 || exit $?
cat gpurun_out/${TAG}_gemm_ab.log | grep -v amdgpu.ids
echo "== bench"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-300
CMHAR_GEMM_PERSIST=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_np.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench_np.log | cut -c1-300
exit 0
