set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python scripts/splitk_sweep.py &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "halo or splitk" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1 && tail -2 gpurun_out/pytest_k.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c150-240
