#!/bin/bash
# The non-headline BASELINE configs through bench.py --workload (same JSON schema), plus the R3D-18 step trace and
# PMC traffic.  usage: tools/gpu_r03_workloads.sh TAG
TAG=${1:-r03w}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
for W in r3d fusion ood_fp16; do
  echo "== $W"
  timeout -k 10 400 python bench.py --workload $W --steps 20 --warmup 5 > gpurun_out/${TAG}_${W}.log 2>&1 || exit $?
  tail -1 gpurun_out/${TAG}_${W}.log | cut -c1-200
done
echo "== r3d trace"
tools/prof_step.sh ${TAG}_r3d --workload r3d || exit $?
echo "== r3d pmc"
CMD="python bench.py --workload r3d --steps 2 --warmup 1 --no-trace"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_r3d_fetch -o run -- \
  python bench.py --workload r3d --steps 2 --warmup 1 --no-trace > gpurun_out/${TAG}_r3d_fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_r3d_write -o run -- \
  python bench.py --workload r3d --steps 2 --warmup 1 --no-trace > gpurun_out/${TAG}_r3d_write.log 2>&1 || exit $?
python tools/pmc_traffic.py gpurun_out/${TAG}_r3d_fetch gpurun_out/${TAG}_r3d_write gpurun_out/${TAG}_r3d_pmc_traffic.json \
  "$(cat .commit 2>/dev/null)" "$CMD" > gpurun_out/${TAG}_r3d_pmc_traffic.txt 2>&1 || exit $?
find gpurun_out/${TAG}_r3d_fetch gpurun_out/${TAG}_r3d_write -name "*.csv" -size +20M -delete
head -12 gpurun_out/${TAG}_r3d_pmc_traffic.txt
exit 0
