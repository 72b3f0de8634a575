#!/bin/bash
# R3D-18 measurement session: kernel trace (--stats), FETCH_SIZE / WRITE_SIZE passes, then the bench line.
# usage: COMMIT=<sha> tools/gpu_r3d_prof.sh TAG   (then copy gpurun_out/TAG_r3d_* into profiles/)
TAG=${1:-r3dq}
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/${TAG}_r3d_prof gpurun_out/${TAG}_r3d_fetch gpurun_out/${TAG}_r3d_write
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_r3d_prof -o run -- \
  python tools/bench_r3d.py --steps 4 --warmup 2 > gpurun_out/${TAG}_r3d_prof.log 2>&1 || exit $?
python tools/kstats.py gpurun_out/${TAG}_r3d_prof > gpurun_out/${TAG}_r3d_kernels.txt || exit $?
find gpurun_out/${TAG}_r3d_prof -name "*kernel_trace.csv" -delete
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_r3d_fetch -o run -- \
  python tools/bench_r3d.py --steps 1 --warmup 1 > gpurun_out/${TAG}_r3d_fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_r3d_write -o run -- \
  python tools/bench_r3d.py --steps 1 --warmup 1 > gpurun_out/${TAG}_r3d_write.log 2>&1 || exit $?
python tools/pmc_traffic.py gpurun_out/${TAG}_r3d_fetch gpurun_out/${TAG}_r3d_write gpurun_out/${TAG}_r3d_pmc.json \
  ${COMMIT:-unknown} "python tools/bench_r3d.py --steps 1 --warmup 1" > gpurun_out/${TAG}_r3d_pmc.txt 2>&1 || exit $?
find gpurun_out/${TAG}_r3d_fetch gpurun_out/${TAG}_r3d_write -name "*.csv" -size +20M -delete
timeout -k 10 300 python tools/bench_r3d.py > gpurun_out/${TAG}_r3d_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_r3d_bench.log | cut -c1-300
exit 0
