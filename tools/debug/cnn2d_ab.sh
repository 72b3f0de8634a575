#!/bin/bash
# Per-frame CNN step (tools/bench_cnn2d.py) with library builds alternated twice.  usage: cnn2d_ab.sh TAG BACKBONE lib...
TAG=$1; BB=$2; shift 2
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS="$PWD/crossmodal-imu-video-ood-har_amd/cmhar/libcmhar.so"
for l in "$@"; do LIBS="$LIBS $PWD/$l"; done
for rep in 1 2; do
  for lib in $LIBS; do
    n=$(basename $lib .so)
    CMHAR_LIB=$lib timeout -k 10 300 python tools/bench_cnn2d.py --video-backbone $BB > gpurun_out/${TAG}_${n}_${rep}.log 2>&1 || exit $?
    echo "$n rep=$rep $(tail -1 gpurun_out/${TAG}_${n}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
exit 0
