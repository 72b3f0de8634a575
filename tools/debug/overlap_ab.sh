#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for ov in 0 1; do
    CMHAR_OVERLAP_WGRAD=$ov timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ov_${ov}_${rep}.log 2>&1 || exit $?
    echo "ov=$ov rep=$rep $(tail -1 gpurun_out/ov_${ov}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["achieved"], d["roofline"].get("frac"))')"
  done
done
