#!/bin/bash
# Round-5 session: bench-step A/B of library variants (alternated), optionally a parity subset and a kernel trace on
# the last variant.  usage: tools/gpu_r05_step_ab.sh TAG lib...   (PARITY_K="pytest -k expr", TRACE=1)
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
last=${@: -1}
if [ -n "$PARITY_K" ]; then
  echo "== parity on $last"
  CMHAR_LIB=$PWD/$last timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread -rf -k "$PARITY_K" > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -gt 1 ] && exit $rc
fi
echo "== step A/B"
bash tools/debug/lib_step_ab.sh ${TAG}_step "$@" || exit $?
if [ -n "$TRACE" ]; then
  echo "== kernel trace on $last"
  CMHAR_LIB=$PWD/$last bash tools/prof_step.sh ${TAG} || exit $?
  tail -20 gpurun_out/${TAG}_kernels.txt
fi
exit 0
