#!/bin/bash
# (The CMHAR_BENCH_STEP_PRIORITY bench knob was measured neutral and removed: profiles/r06_step_priority_ab.log, DESIGN.md.)
# A/B: the bench step on a high-priority stream (CMHAR_BENCH_STEP_PRIORITY=-1, the IMU side stream at the default
# priority below it) vs the default stream, alternated on one box; headline workload and R3D-18 (config 2).
export TMPDIR=/tmp CMHAR_BENCH_PEAK_PROBE=0
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/prio_ab.log
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())" | tee $OUT
for rep in 1 2; do
  for p in default -1; do
    envs=""; [ $p != default ] && envs="CMHAR_BENCH_STEP_PRIORITY=$p"
    line=$(env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace 2>>gpurun_out/prio_ab_err.log | tail -1) || exit $?
    echo "videomae prio=$p rep=$rep $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $OUT
  done
done
