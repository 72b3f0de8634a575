#!/bin/bash
# The bench step under alternative environment settings, alternated twice.  usage: env_step_ab.sh TAG 'A=0' 'A=1' …
TAG=$1; shift
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for kv in "$@"; do
    n=$(echo "$kv" | tr -c 'A-Za-z0-9_\n' '_')
    env $kv timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline \
      > gpurun_out/${TAG}_${n}_${rep}.log 2>&1 || exit $?
    echo "$kv rep=$rep $(tail -1 gpurun_out/${TAG}_${n}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels"]; print(d["value"], d["ms_per_step"], {a: b["ms_per_step"] for a, b in k.items()})')"
  done
done
exit 0
