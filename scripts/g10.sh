set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -q -x -k "attention or fft or trajectory" > gpurun_out/t_attn.log 2>&1 || { tail -40 gpurun_out/t_attn.log; exit 1; }
tail -1 gpurun_out/t_attn.log
timeout -k 10 300 python scripts/attn_bench.py
