#!/bin/bash
# hipBLASLt kernel names / times on the step's GEMM shapes (tools/debug/blaslt_shapes.py) under rocprofv3
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/debug/blaslt_shapes.py > gpurun_out/blaslt_shapes.log 2>&1 || exit 1
cat gpurun_out/blaslt_shapes.log | grep -v amdgpu.ids
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/blaslt_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/debug/blaslt_shapes.py > $GRAFT_REPO_ROOT/gpurun_out/blaslt_prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && find gpurun_out/blaslt_prof -name '*kernel_stats.csv' | head -1 | xargs -I{} python3 -c "
import csv,sys
for r in csv.DictReader(open('{}')):
    print(r['Name'][:400], r['Calls'], r['AverageNs'])
"
