#!/bin/bash
# Round-5 A/B of library builds on the R3D-18 path: conv kernel times per layer (tools/debug/conv_bench.py) per
# build, then the R3D-18 step alternated twice.  The in-tree library is the 'cur' arm.
# usage: tools/gpu_r05_libab.sh TAG LAYERS lib.so...
TAG=$1; LAYERS=$2; shift 2
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS="$PWD/crossmodal-imu-video-ood-har_amd/cmhar/libcmhar.so"
for l in "$@"; do LIBS="$LIBS $PWD/$l"; done
for lib in $LIBS; do
  n=$(basename $lib .so)
  CMHAR_LIB=$lib timeout -k 10 200 python tools/debug/conv_bench.py --layers $LAYERS --reps 20 \
    > gpurun_out/${TAG}_conv_$n.log 2>&1 || exit $?
  echo "== $n"; grep -v amdgpu.ids gpurun_out/${TAG}_conv_$n.log
done
for rep in 1 2; do
  for lib in $LIBS; do
    n=$(basename $lib .so)
    CMHAR_LIB=$lib timeout -k 10 300 python bench.py --workload r3d --steps 30 --warmup 5 --no-cpu-baseline \
      > gpurun_out/${TAG}_r3d_${n}_${rep}.log 2>&1 || exit $?
    echo "$n rep=$rep $(tail -1 gpurun_out/${TAG}_r3d_${n}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
exit 0
