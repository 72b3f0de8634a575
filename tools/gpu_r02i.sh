mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py tests/test_models_gpu.py tests/test_fusion_gpu.py tests/test_geometries_gpu.py -q -p no:cacheprovider --timeout 180 --timeout-method thread -rf > gpurun_out/r02i_pytest.log 2>&1; rc=$?; tail -4 gpurun_out/r02i_pytest.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02i_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r02i_bench.log | cut -c1-300
