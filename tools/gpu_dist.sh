set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread > gpurun_out/dist_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u tools/bench_dist_chol.py > gpurun_out/dist_chol.log 2>&1
echo ok bench
