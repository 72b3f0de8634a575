#!/bin/bash
# Measurement session: PMC traffic (FETCH_SIZE / WRITE_SIZE passes), PMC MFMA utilisation, kernel trace, then the
# bench (with the CPU baseline) reading the PMC summaries of this same build (profiles/ROUND_pmc_*.json, the files
# bench.py's TRAFFIC_JSON / MFMA_JSON name).
# usage: tools/gpu_prof.sh TAG COMMIT ROUND   (then copy gpurun_out/TAG_{pmc_*,kernels.txt,bench.log} into profiles/)
TAG=${1:-r04}
COMMIT=${2:-unknown}
ROUND=${3:-r04}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
CMD="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-trace"
echo "== pmc traffic"
rm -rf gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write gpurun_out/${TAG}_mfma
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_fetch -o run -- \
  python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-trace > gpurun_out/${TAG}_fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_write -o run -- \
  python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-trace > gpurun_out/${TAG}_write.log 2>&1 || exit $?
# written under gpurun_out/ (merged back) AND into profiles/ (read by the bench below on the box)
python tools/pmc_traffic.py gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write gpurun_out/${TAG}_pmc_traffic.json \
  "$COMMIT" "$CMD" > gpurun_out/${TAG}_pmc_traffic_top.txt 2>&1 || exit $?
cp gpurun_out/${TAG}_pmc_traffic.json profiles/${ROUND}_pmc_traffic.json
echo "== pmc mfma"
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA --kernel-trace \
  --output-format csv -d gpurun_out/${TAG}_mfma -o run -- \
  python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-trace > gpurun_out/${TAG}_mfma.log 2>&1 || exit $?
python tools/pmc_mfma.py gpurun_out/${TAG}_mfma gpurun_out/${TAG}_pmc_mfma.json "$COMMIT" "$CMD" \
  > gpurun_out/${TAG}_pmc_mfma_top.txt 2>&1 || exit $?
cp gpurun_out/${TAG}_pmc_mfma.json profiles/${ROUND}_pmc_mfma.json
find gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write gpurun_out/${TAG}_mfma -name "*.csv" -size +20M -delete
echo "== kernel trace"
tools/prof_step.sh ${TAG} || exit $?
echo "== bench"
timeout -k 10 900 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-300
exit 0
