mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_cnn2d_gpu.py tests/test_r3d_gpu.py -q -s -p no:cacheprovider --timeout 180 --timeout-method thread -rf > gpurun_out/r02j_pytest.log 2>&1; rc=$?; tail -4 gpurun_out/r02j_pytest.log; grep worst gpurun_out/r02j_pytest.log | cut -c1-300; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/bench_cnn2d.py --video-backbone resnet18 > gpurun_out/r02j_resnet.log 2>&1 || exit $?
tail -1 gpurun_out/r02j_resnet.log
timeout -k 10 300 python tools/bench_cnn2d.py --video-backbone mobilenet_v2 > gpurun_out/r02j_mobilenet.log 2>&1 || exit $?
tail -1 gpurun_out/r02j_mobilenet.log
rm -rf gpurun_out/r02j_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02j_prof -o run -- python tools/bench_cnn2d.py --video-backbone mobilenet_v2 --steps 3 --warmup 2 > gpurun_out/r02j_prof.log 2>&1 || exit $?
python tools/rocpd_summary.py gpurun_out/r02j_prof/run_results.db > gpurun_out/r02j_mobilenet_kernels.txt 2>&1; head -24 gpurun_out/r02j_mobilenet_kernels.txt | cut -c1-70,100-150
