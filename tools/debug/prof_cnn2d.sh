#!/bin/bash
# rocprofv3 kernel trace of the MobileNetV2 per-frame step (tools/bench_cnn2d.py) -> gpurun_out/s2t_kernels.txt
set -o pipefail
export TMPDIR=/tmp
rm -rf gpurun_out/s2t_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s2t_prof -o run -- python tools/bench_cnn2d.py --video-backbone mobilenet_v2 --steps 4 --warmup 2 > gpurun_out/s2t_prof.log 2>&1 || exit $?
python tools/kstats.py gpurun_out/s2t_prof > gpurun_out/s2t_kernels.txt || exit $?
find gpurun_out/s2t_prof -name "*kernel_trace.csv" -delete
head -25 gpurun_out/s2t_kernels.txt | cut -c1-140
