set -o pipefail
echo NEW; timeout -k 10 120 python scripts/bn_bench.py &&
echo OLD; FS2HIP_LIB=$PWD/ablib/libfs2hip_old.so timeout -k 10 120 python scripts/bn_bench.py &&
echo NEW; timeout -k 10 120 python scripts/bn_bench.py &&
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "batchnorm or bn or postnet or parity" > gpurun_out/pytest_bn.log 2>&1 && tail -1 gpurun_out/pytest_bn.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c150-240
