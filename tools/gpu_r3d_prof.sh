set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r3dq
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3dq -o run -- python tools/bench_r3d.py --steps 4 --warmup 2 > gpurun_out/r3dq.log 2>&1 || exit $?
find gpurun_out/r3dq -name "*kernel_trace.csv" -delete
rm -rf gpurun_out/r3dq_fetch gpurun_out/r3dq_write
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3dq_fetch -o run -- python tools/bench_r3d.py --steps 1 --warmup 1 > gpurun_out/r3dq_fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r3dq_write -o run -- python tools/bench_r3d.py --steps 1 --warmup 1 > gpurun_out/r3dq_write.log 2>&1 || exit $?
python tools/pmc_traffic.py gpurun_out/r3dq_fetch gpurun_out/r3dq_write gpurun_out/r3dq_pmc.json ${COMMIT:-unknown} "python tools/bench_r3d.py --steps 1 --warmup 1" > gpurun_out/r3dq_pmc.txt 2>&1
find gpurun_out/r3dq_fetch gpurun_out/r3dq_write -name "*.csv" -size +20M -delete
