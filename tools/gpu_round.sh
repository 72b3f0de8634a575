#!/bin/bash
# One GPU session: parity tests, smoke, short bench.  Stops at the first crash-like exit status.
# usage: tools/gpu_round.sh TAG [bench-args...]
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 -rf > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/${TAG}_pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a gpurun_out/${TAG}_smoke.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py "$@" > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc" | tee -a gpurun_out/${TAG}_bench.log
exit $rc
