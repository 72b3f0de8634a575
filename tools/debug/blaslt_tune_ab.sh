#!/bin/bash
# (The CMHAR_BLASLT_TUNE first-use timing it compares measured neutral and was removed: profiles/r06_blaslt_tune_ab.log.)
# hipBLASLt first-use candidate timing A/B (round 6): tests/test_blaslt_gpu.py, then the bench step alternated between
# the heuristic's first choice (CMHAR_BLASLT_TUNE=0) and the fastest of its top 8 timed on first use (default).
export TMPDIR=/tmp CMHAR_BENCH_PEAK_PROBE=0
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/blaslt_tune_ab.log
timeout -k 10 300 python -u -m pytest tests/test_blaslt_gpu.py -q -x -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/blaslt_tune_tests.log 2>&1; rc=$?
tail -1 gpurun_out/blaslt_tune_tests.log | tee $OUT
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for t in 0 1; do
    line=$(CMHAR_BLASLT_TUNE=$t timeout -k 10 300 python bench.py --no-cpu-baseline 2>>gpurun_out/blaslt_tune_err.log | tail -1) || exit $?
    echo "tune=$t rep=$rep $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d.get("kernels",{}); print(d["value"], d["ms_per_step"], k.get("hipblaslt_linear"))')" | tee -a $OUT
  done
done
