#!/bin/bash
# Round-5 A/B of one library knob on the R3D-18 path: conv kernel times per layer (tools/debug/conv_bench.py), then
# the R3D-18 step alternated twice, VAR=A vs VAR=B; then the R3D conv tests at the default.
# usage: tools/gpu_r05_envab.sh TAG VAR A B [LAYERS]
TAG=$1; VAR=$2; A=$3; B=$4; LAYERS=${5:-layer1,layer2,layer3}
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in $A $B; do
  env $VAR=$m timeout -k 10 200 python tools/debug/conv_bench.py --layers $LAYERS --reps 20 \
    > gpurun_out/${TAG}_conv_$m.log 2>&1 || exit $?
  echo "$VAR=$m"; grep -v amdgpu.ids gpurun_out/${TAG}_conv_$m.log
done
for rep in 1 2; do
  for m in $A $B; do
    env $VAR=$m timeout -k 10 300 python bench.py --workload r3d --steps 30 --warmup 5 --no-cpu-baseline \
      > gpurun_out/${TAG}_r3d_${m}_${rep}.log 2>&1 || exit $?
    echo "$VAR=$m rep=$rep $(tail -1 gpurun_out/${TAG}_r3d_${m}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_r3d_production_gpu.py tests/test_r3d_gpu.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/${TAG}_r3d_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_r3d_tests.log; exit $rc
