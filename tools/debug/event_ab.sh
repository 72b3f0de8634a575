#!/bin/bash
# (The fence-free event variant this script compares was measured and reverted: profiles/r06_event_fence_ab.log, DESIGN.md.)
# A/B of the bench's timed-loop event bracketing (round 6): fence-free libcmhar events (default) vs torch.cuda.Event
# vs no bracketing at all (--no-trace), alternated on one box; then a kernel trace of the default to read the gaps.
export TMPDIR=/tmp CMHAR_BENCH_PEAK_PROBE=0
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/event_ab.log
: > $OUT
for rep in 1 2; do
  for mode in nofence torch notrace; do
    extra=""; envs=""
    [ $mode = torch ] && envs="CMHAR_TRACE_EVENT_FLAGS=torch"
    [ $mode = notrace ] && extra="--no-trace"
    line=$(env $envs timeout -k 10 300 python bench.py --no-cpu-baseline $extra 2>gpurun_out/event_ab_err.log | tail -1) || exit $?
    echo "$mode rep=$rep $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d.get("roofline") or {}; print(d["value"], d["ms_per_step"], r.get("avg_launch_ms"), r.get("frac"))')" | tee -a $OUT
  done
done
bash tools/prof_step.sh evab || exit $?
grep -n "inter-kernel gaps\|steady state" gpurun_out/evab_kernels.txt | tee -a $OUT
