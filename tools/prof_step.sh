#!/bin/bash
# rocprofv3 kernel trace of a short bench run → per-kernel summary.  tools/prof_step.sh TAG [bench args...]
export TMPDIR=/tmp
TAG=$1; shift
rm -rf gpurun_out/${TAG}_prof
# (the bench's MFMA peak probe off: its 4 launches of ~30 ms would dominate the per-kernel table)
export CMHAR_BENCH_PEAK_PROBE=0
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
  python bench.py --steps 4 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
CMHAR_KSTATS_CONTEXT=${CMHAR_KSTATS_CONTEXT:-FillFunctor,copyBuffer,colsum_rows2} python tools/kstats.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_kernels.txt
find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" -delete
tail -3 gpurun_out/${TAG}_kernels.txt
