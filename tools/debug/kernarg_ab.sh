#!/bin/bash
# The bench step with kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs the runtime default, alternated.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in 1 0; do
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-trace \
      > gpurun_out/kargs_${v}_${rep}.log 2>&1 || exit $?
    echo "DEV_KERNARG=$v rep=$rep $(tail -1 gpurun_out/kargs_${v}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
exit 0
