#!/bin/bash
# Round-4 parity session: R3D-18 per-layer bf16 diagnosis, then the bf16 parity tests of R3D-18 / CNNs / fusion / DP.
# usage: tools/gpu_r04_parity.sh TAG [pytest -k expression]
TAG=${1:-r04p}
KEXPR=${2:-"bf16 or fusion or dataparallel"}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
echo "== dgrad layout A/B"
timeout -k 10 240 python -u tools/debug/dgrad_layout_ab.py > gpurun_out/${TAG}_dgrad_ab.log 2>&1 || exit $?
cat gpurun_out/${TAG}_dgrad_ab.log
if [ -f var/libA.so ] && [ -f var/libB.so ]; then
  echo "== attention A/B (var/libA.so vs var/libB.so)"
  timeout -k 10 300 python -u tools/debug/attn_ab.py var/libA.so var/libB.so var/libC.so var/libD.so var/libE.so var/libF.so --prescaled > gpurun_out/${TAG}_attn_ab.log 2>&1 || exit $?
  cat gpurun_out/${TAG}_attn_ab.log
fi
echo "== r3d layers"
timeout -k 10 300 python -u tools/debug/r3d_bf16_layers.py > gpurun_out/${TAG}_r3d_layers.log 2>&1 || exit $?
tail -20 gpurun_out/${TAG}_r3d_layers.log
echo "== tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -rf -k "$KEXPR" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_pytest.log; exit $rc
