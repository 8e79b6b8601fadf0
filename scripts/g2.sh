# full GPU check: kernel + parity tests, smoke, GEMM micro-bench, bench, kernel profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 120 python scripts/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
bash scripts/prof.sh ${1:-r1d}
