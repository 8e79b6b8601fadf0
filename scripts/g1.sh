set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -k "conv" > gpurun_out/t_conv.log 2>&1 || { tail -40 gpurun_out/t_conv.log; exit 1; }
tail -2 gpurun_out/t_conv.log
echo OLD; FS2_GEMM_OLD=1 timeout -k 10 120 python scripts/gemm_bench.py
echo NEW-W2; timeout -k 10 120 python scripts/gemm_bench.py
echo NEW-W1; FS2_WGRAD_STAGES=1 timeout -k 10 120 python scripts/gemm_bench.py
