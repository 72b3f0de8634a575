#!/bin/bash
# Kernel traces of the bench step per library build (CMHAR_LIB), kept as CSV for a per-launch comparison
# (tools/debug/trace_cmp.py).  usage: trace_ab.sh TAG lib.so...
TAG=$1; shift
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in "$@"; do
  n=$(basename $lib .so)
  rm -rf gpurun_out/${TAG}_${n}
  CMHAR_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_${n} -o run -- \
    python bench.py --steps 4 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_${n}.log 2>&1 || exit $?
  tail -1 gpurun_out/${TAG}_${n}.log | cut -c1-200
done
exit 0
