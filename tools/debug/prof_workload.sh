#!/bin/bash
# rocprofv3 kernel trace of one bench tool's step -> gpurun_out/TAG_kernels.txt
# usage: tools/debug/prof_workload.sh TAG tools/bench_fusion.py [args...]
TAG=$1; shift
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/${TAG}_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python "$@" \
  > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
python tools/kstats.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_kernels.txt || exit $?
find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" -delete
head -30 gpurun_out/${TAG}_kernels.txt | cut -c1-140
