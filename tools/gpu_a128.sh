# flavor-A 128-drone envs on the GPU box: the parity / stats cases, then a short a128 bench
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity_a.py tests/test_gpu_stats.py -k "128 or flavor_a_episode" -v --timeout 300 --timeout-method thread > gpurun_out/a128_tests.log 2>&1
rc=$?
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --config a128 --steps 200 --no-cpu-baseline --e2e-iters 0 > gpurun_out/a128_bench.log 2>&1
