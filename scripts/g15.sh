set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -2 gpurun_out/pytest_gpu.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c150-240 &&
timeout -k 10 300 python bench_infer.py > gpurun_out/binfer.log 2>&1 && tail -1 gpurun_out/binfer.log | cut -c1-300
