#!/bin/bash
# Round-5 A/B of the nine-tap forward on Cout > 64 (layers 2-3 forward and flipped dgrad): conv kernel times per
# layer, then the R3D-18 step, CMHAR_FWD_ROWS3=1 (layer 1 only, the round-4 plan) vs default (all Cout % 64),
# alternated; then the R3D conv tests.  usage: tools/gpu_r05_rows3.sh TAG
TAG=$1
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 1 2; do
  CMHAR_FWD_ROWS3=$m CMHAR_WGRAD_ROWS3=$m timeout -k 10 200 python tools/debug/conv_bench.py --layers layer1,layer2,layer3 --reps 20 \
    > gpurun_out/${TAG}_conv_m$m.log 2>&1 || exit $?
  echo "mode $m"; cat gpurun_out/${TAG}_conv_m$m.log
done
for rep in 1 2; do
  for m in 1 2; do
    CMHAR_FWD_ROWS3=$m CMHAR_WGRAD_ROWS3=$m timeout -k 10 300 python bench.py --workload r3d --steps 30 --warmup 5 --no-cpu-baseline \
      > gpurun_out/${TAG}_r3d_m${m}_${rep}.log 2>&1 || exit $?
    echo "mode $m rep=$rep $(tail -1 gpurun_out/${TAG}_r3d_m${m}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_r3d_production_gpu.py tests/test_r3d_gpu.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/${TAG}_r3d_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_r3d_tests.log; exit $rc
