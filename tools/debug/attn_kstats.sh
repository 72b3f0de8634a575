#!/bin/bash
# Per-kernel rocprofv3 stats of the flash attention forward + pre-scaled backward (tools/debug/attn_once.py) for
# each library build given.   usage: tools/debug/attn_kstats.sh TAG lib1.so [lib2.so ...]
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in "$@"; do
  n=$(basename $lib .so)
  rm -rf gpurun_out/${TAG}_${n}_ks
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${n}_ks -o run -- \
    python tools/debug/attn_once.py $lib --reps 10 > gpurun_out/${TAG}_${n}_ks.log 2>&1 || exit $?
  echo "== $n"
  python tools/kstats.py gpurun_out/${TAG}_${n}_ks | head -8 | cut -c1-60,100-160
  find gpurun_out/${TAG}_${n}_ks -name "*kernel_trace.csv" -delete
done
