set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -1 gpurun_out/pytest_gpu.log &&
bash scripts/prof.sh r1i && python scripts/kshape.py $(find gpurun_out/prof_r1i -name "*kernel_trace.csv" | head -1) 7 80 > gpurun_out/shapes_r1i.txt && grep -E "ln_bwd|ROOFLINE|kernel time" gpurun_out/shapes_r1i.txt
