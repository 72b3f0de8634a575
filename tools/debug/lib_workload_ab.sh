#!/bin/bash
# bench.py --workload W with alternative library builds (CMHAR_LIB), alternated twice.
# usage: lib_workload_ab.sh TAG WORKLOAD lib...
TAG=$1; W=$2; shift 2
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    CMHAR_LIB=$PWD/$lib timeout -k 10 300 python bench.py --workload $W --steps 30 --warmup 5 --no-cpu-baseline \
      > gpurun_out/${TAG}_${n}_${rep}.log 2>&1 || exit $?
    echo "$n rep=$rep $(tail -1 gpurun_out/${TAG}_${n}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
exit 0
