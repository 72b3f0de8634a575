#!/bin/bash
# Full measurement session on one GPU: parity tests, smoke, bench (with CPU baseline), rocprofv3 kernel-trace summary of
# a short bench run, and two PMC passes (FETCH_SIZE / WRITE_SIZE) that give per-kernel HBM traffic.
# usage: tools/gpu_full.sh TAG [COMMIT]    (outputs under gpurun_out/TAG_*; COMMIT = the git hash of the tree sent)
TAG=${1:-full}
COMMIT=${2:-unknown}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
step() { echo "== $1"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -gt 1 ] && exit $rc
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_smoke.log
step pmc
rm -rf gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_fetch -o run -- \
  python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-trace > gpurun_out/${TAG}_fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_write -o run -- \
  python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-trace > gpurun_out/${TAG}_write.log 2>&1 || exit $?
python tools/pmc_traffic.py gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write gpurun_out/${TAG}_pmc_traffic.json \
  "$COMMIT" "python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-trace" \
  > gpurun_out/${TAG}_pmc_traffic.txt 2>&1 || exit $?
# the bench below reads the traffic of this same build
cp gpurun_out/${TAG}_pmc_traffic.json profiles/r02_pmc_traffic.json
find gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write -name "*.csv" -size +20M -delete
step prof
rm -rf gpurun_out/${TAG}_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- \
  python bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" -delete
step bench
timeout -k 10 900 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log
exit 0
