#!/bin/bash
# GPU test session: full GPU test suite (-s: the bf16 tests print their worst per-parameter errors), smoke, and a
# short bench.  usage: tools/gpu_tests.sh TAG [pytest -k expression]
TAG=${1:-r04}
KEXPR=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
echo "== tests"
if [ -n "$KEXPR" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -rf -k "$KEXPR" > gpurun_out/${TAG}_pytest.log 2>&1
else
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -rf > gpurun_out/${TAG}_pytest.log 2>&1
fi
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -gt 1 ] && exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_smoke.log
echo "== bench"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
exit 0
