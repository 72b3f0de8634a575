#!/bin/bash
# hipBLASLt routing for the fp16 inference path (config 5, round 6): tests, then the fp16 OOD streams alternated
# between the hand-written kernels (CMHAR_BLASLT="") and the default routing list.
export TMPDIR=/tmp CMHAR_BENCH_PEAK_PROBE=0
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/blaslt_fp16_ab.log
timeout -k 10 400 python -u -m pytest tests/test_blaslt_gpu.py tests/test_fp16_gpu.py -q -x -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/blaslt_fp16_tests.log 2>&1; rc=$?
tail -1 gpurun_out/blaslt_fp16_tests.log | tee $OUT
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in none default; do
    if [ $v = none ]; then export CMHAR_BLASLT=""; else unset CMHAR_BLASLT; fi
    for m in siglip fusion; do
      extra=""; [ $m = fusion ] && extra="--model fusion"
      line=$(timeout -k 10 300 python tools/bench_ood.py $extra 2>>gpurun_out/blaslt_fp16_err.log | tail -1) || exit $?
      echo "blaslt=$v model=$m rep=$rep $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("ms_per_step"))')" | tee -a $OUT
    done
  done
done
