set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -k "conv" > gpurun_out/t_conv.log 2>&1 || { tail -40 gpurun_out/t_conv.log; exit 1; }
tail -1 gpurun_out/t_conv.log
timeout -k 10 400 python scripts/nt_sweep.py
timeout -k 10 500 python scripts/wgrad_sweep.py
