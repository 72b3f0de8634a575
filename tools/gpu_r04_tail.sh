#!/bin/bash
# Round-4 tail-stream session: the flash kernels' ragged tails on a second stream (product build) against
# var/libB.so (-DCMHAR_ATTN_TAIL_STREAM_DEFAULT=0) in one process, the attention / model tests, and the step both ways.
# usage: tools/gpu_r04_tail.sh TAG
TAG=${1:-r04t}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
echo "== tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
  -k "attention or flash or videomae or token0 or peak_probe or fusion or threading" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_pytest.log; [ $rc -gt 1 ] && exit $rc
grep "MFMA peak probe" gpurun_out/${TAG}_pytest.log
echo "== attention A/B (A = tails on a side stream, B = one stream)"
timeout -k 10 300 python -u tools/debug/attn_ab.py crossmodal-imu-video-ood-har_amd/cmhar/libcmhar.so var/libB.so --prescaled \
  > gpurun_out/${TAG}_attn_ab.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${TAG}_attn_ab.log
echo "== bench"
for v in 1 0 1 0; do
  CMHAR_ATTN_TAIL_STREAM=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_$v.log 2>&1 || exit $?
  echo "tail_stream=$v $(tail -1 gpurun_out/${TAG}_bench_$v.log | cut -c1-200)"
done
exit 0
