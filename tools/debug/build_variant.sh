#!/bin/bash
# Build a libcmhar.so variant for in-process A/B runs (tools/debug/*_ab.py).
# usage: tools/debug/build_variant.sh OUT.so [GIT_REV|-] [extra hipcc flags...]
#   GIT_REV: build the csrc/ + include/ of that commit ('-' = the working tree)
set -e
OUT=$1; REV=${2:--}; shift 2 || true
REPO=$(cd "$(dirname "$0")/../.." && pwd)
TMP=$(mktemp -d)
mkdir -p $TMP/csrc $TMP/include
if [ "$REV" = "-" ]; then
  cp $REPO/crossmodal-imu-video-ood-har_amd/csrc/* $TMP/csrc/; cp $REPO/include/cmhar.h $TMP/include/
else
  for f in $(git -C $REPO ls-tree --name-only $REV crossmodal-imu-video-ood-har_amd/csrc/); do
    git -C $REPO show $REV:$f > $TMP/csrc/$(basename $f); done
  git -C $REPO show $REV:include/cmhar.h > $TMP/include/cmhar.h
fi
objs=""
for f in $TMP/csrc/*.hip; do
  o=$TMP/$(basename $f .hip).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -I$TMP/include "$@" -c $f -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT $objs
rm -rf $TMP
echo built $OUT
