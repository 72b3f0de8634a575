#!/bin/bash
# Per-step cost of the data-parallel machinery on one GPU: bench.py with the reducer's full bucket / RCCL protocol in
# a one-rank group (CMHAR_BENCH_REDUCE_SINGLE=1) vs without, alternated twice, for the given workloads.
# usage: tools/debug/dp_cost.sh TAG workload...
TAG=$1; shift
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for W in "$@"; do
  for rep in 1 2; do
    for v in 0 1; do
      CMHAR_BENCH_REDUCE_SINGLE=$v timeout -k 10 300 python bench.py --workload $W --steps 30 --warmup 5 --no-cpu-baseline \
        > gpurun_out/${TAG}_${W}_${v}_${rep}.log 2>&1 || exit $?
      echo "$W reduce_single=$v rep=$rep $(tail -1 gpurun_out/${TAG}_${W}_${v}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
exit 0
