#!/bin/bash
# One GPU session: parity tests, smoke, bench, optional rocprofv3 kernel-trace summary of a short bench.
# Stops at the first crash-like exit status (anything other than 0 / 1).
# usage: tools/gpu_round.sh TAG [--tests] [--smoke] [--bench "args"] [--prof "args"]
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
while [ $# -gt 0 ]; do
  case "$1" in
    --tests)
      timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 -rf > gpurun_out/${TAG}_pytest.log 2>&1
      rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/${TAG}_pytest.log; tail -3 gpurun_out/${TAG}_pytest.log
      [ $rc -gt 1 ] && exit $rc; shift;;
    --smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc" | tee -a gpurun_out/${TAG}_smoke.log
      [ $rc -gt 1 ] && exit $rc; shift;;
    --bench)
      timeout -k 10 900 python bench.py $2 > gpurun_out/${TAG}_bench.log 2>&1
      rc=$?; echo "bench rc=$rc" | tee -a gpurun_out/${TAG}_bench.log; tail -c 3000 gpurun_out/${TAG}_bench.log
      [ $rc -ne 0 ] && exit $rc; shift 2;;
    --prof)
      rm -rf gpurun_out/${TAG}_prof
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python bench.py $2 \
        > gpurun_out/${TAG}_prof.log 2>&1
      rc=$?; echo "prof rc=$rc" | tee -a gpurun_out/${TAG}_prof.log
      find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" -exec head -40 {} \; > gpurun_out/${TAG}_kernel_stats.txt 2>/dev/null
      find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" -exec rm -f {} \; 2>/dev/null
      [ $rc -ne 0 ] && exit $rc; shift 2;;
    *) echo "unknown arg $1"; exit 2;;
  esac
done
exit 0
