#!/bin/bash
# The other BASELINE configs through their bench tools on one GPU, each its own JSON line under gpurun_out/TAG_*.json:
# fusion (config 4 per GPU), R3D-18 (config 2's backbone), fp16 OOD stream (config 5, SigLIP and fusion heads),
# ResNet-18 / MobileNetV2 per-frame backbones, and the bench step at config 4's VideoMAE geometry.
TAG=${1:-cfg}
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 300 python "$@" > gpurun_out/${TAG}_${name}.log 2>&1 || exit $?;
        tail -1 gpurun_out/${TAG}_${name}.log > gpurun_out/${TAG}_${name}.json; echo "$name: $(cut -c1-160 gpurun_out/${TAG}_${name}.json)"; }
run fusion tools/bench_fusion.py
run r3d tools/bench_r3d.py
run ood_fp16 tools/bench_ood.py
run ood_fusion_fp16 tools/bench_ood.py --model fusion
run resnet18 tools/bench_cnn2d.py --video-backbone resnet18
run mobilenet_v2 tools/bench_cnn2d.py --video-backbone mobilenet_v2
run bench_32f tools/../bench.py --frames 32 --imu-len 400 --batch 8 --steps 10 --warmup 3 --no-cpu-baseline --no-trace
exit 0
