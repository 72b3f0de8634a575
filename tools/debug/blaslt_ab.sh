#!/bin/bash
# hipBLASLt routing A/B (round 6): tests/test_blaslt_gpu.py, then the bench step alternated between the hand-written
# plans (CMHAR_BLASLT unset) and hipBLASLt for the listed N,K shapes, one box; then a traced warm-up breakdown.
export TMPDIR=/tmp CMHAR_BENCH_PEAK_PROBE=0
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/blaslt_ab.log
timeout -k 10 300 python -u -m pytest tests/test_blaslt_gpu.py -q -x -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/blaslt_tests.log 2>&1; rc=$?
tail -3 gpurun_out/blaslt_tests.log | tee $OUT
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in none "768,768" "768,768;768,3072;768,2304;768,1536"; do
    envs=""; [ "$v" != none ] && envs="CMHAR_BLASLT=$v"
    line=$(env $envs timeout -k 10 300 python bench.py --no-cpu-baseline 2>>gpurun_out/blaslt_ab_err.log | tail -1) || exit $?
    echo "blaslt=$v rep=$rep $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d.get("kernels",{}); print(d["value"], d["ms_per_step"], {n: (v["launches"], v["ms_per_step"]) for n, v in k.items() if "blaslt" in n or "gemm8p_kernel<true" in n or "gemm256" in n})')" | tee -a $OUT
  done
done
