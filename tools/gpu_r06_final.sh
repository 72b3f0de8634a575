#!/bin/bash
# Round-6 measurement session on one GPU: every GPU parity test, smoke, the PMC passes the bench line reads
# (FETCH_SIZE / WRITE_SIZE → profiles/r06_pmc_traffic.json, MFMA busy → profiles/r06_pmc_mfma.json), the kernel-trace
# table of a short bench, the bench itself (CPU baseline included) and the fp32 parity-mode bench at B = 32.
# usage: tools/gpu_r06_final.sh TAG COMMIT [--no-tests]   (results under gpurun_out/; copy them to profiles/ after)
TAG=${1:-r06f}
COMMIT=${2:-unknown}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
CMD="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-trace"
if [ "$3" != "--no-tests" ]; then
  echo "== tests"
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 --timeout-method thread -rf \
    > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -gt 1 ] && exit $rc
  echo "== smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
  tail -1 gpurun_out/${TAG}_smoke.log
fi
echo "== pmc traffic"
rm -rf gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write gpurun_out/${TAG}_mfma
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_fetch -o run -- \
  $CMD > gpurun_out/${TAG}_fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_write -o run -- \
  $CMD > gpurun_out/${TAG}_write.log 2>&1 || exit $?
python tools/pmc_traffic.py gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write profiles/r06_pmc_traffic.json "$COMMIT" "$CMD" \
  > profiles/r06_pmc_traffic_top.txt 2>&1 || exit $?
cp profiles/r06_pmc_traffic.json profiles/r06_pmc_traffic_top.txt gpurun_out/   # (profiles/ does not travel back)
echo "== pmc mfma"
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA --kernel-trace --output-format csv \
  -d gpurun_out/${TAG}_mfma -o run -- $CMD > gpurun_out/${TAG}_mfma.log 2>&1 || exit $?
python tools/pmc_mfma.py gpurun_out/${TAG}_mfma profiles/r06_pmc_mfma.json "$COMMIT" "$CMD" \
  > profiles/r06_pmc_mfma_top.txt 2>&1 || exit $?
cp profiles/r06_pmc_mfma.json profiles/r06_pmc_mfma_top.txt gpurun_out/
find gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write gpurun_out/${TAG}_mfma -name "*.csv" -size +20M -delete
echo "== kernel trace"
bash tools/prof_step.sh ${TAG} || exit $?
echo "== bench"
timeout -k 10 900 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log
echo "== bench fp32 (parity mode), B = 32"
timeout -k 10 900 python bench.py --dtype fp32 --batch 32 --steps 10 --warmup 3 --no-cpu-baseline \
  > gpurun_out/${TAG}_bench_fp32.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench_fp32.log
exit 0
