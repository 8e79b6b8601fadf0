set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -3 gpurun_out/pytest_gpu.log &&
timeout -k 10 120 python scripts/ln_bench.py &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c1-400 &&
bash scripts/prof.sh r1g && python scripts/kshape.py $(ls gpurun_out/prof_r1g/*/*kernel_trace.csv 2>/dev/null || find gpurun_out/prof_r1g -name "*kernel_trace.csv" | head -1) 7 30 > gpurun_out/shapes_r1g.txt; cat gpurun_out/shapes_r1g.txt
