#!/bin/bash
# Round-5 session: attention variants A/B + the flash parity tests on one variant library.
# usage: tools/gpu_r05_attn2.sh TAG TESTLIB libA.so libB.so [...]
TAG=$1; TESTLIB=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
echo "== flash tests on $TESTLIB"
CMHAR_LIB=$PWD/$TESTLIB timeout -k 10 400 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 \
  --timeout-method thread -rf -k "flash" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_pytest.log; [ $rc -gt 1 ] && exit $rc
echo "== attn A/B"
timeout -k 10 400 python tools/debug/attn_ab.py "$@" --prescaled --rounds 9 > gpurun_out/${TAG}_attn_ab.log 2>&1 || exit $?
cat gpurun_out/${TAG}_attn_ab.log
exit 0
