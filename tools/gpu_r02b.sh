mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_fp16_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py -q -s -p no:cacheprovider --timeout 180 --timeout-method thread -rf > gpurun_out/r02b_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r02b_pytest.log; grep "fp16 g5" gpurun_out/r02b_pytest.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/bench_ood.py > gpurun_out/r02b_ood.log 2>&1 || exit $?
tail -1 gpurun_out/r02b_ood.log
timeout -k 10 300 python tools/bench_ood.py --model fusion > gpurun_out/r02b_ood_fusion.log 2>&1 || exit $?
tail -1 gpurun_out/r02b_ood_fusion.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02b_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r02b_bench.log | cut -c1-400
