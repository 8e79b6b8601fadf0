# round-end measurement set: default bench line (PMC traffic + CPU baseline), kernel-trace
# summary of a short bench run, per-shape table
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python bench.py > gpurun_out/bench_final.log 2>&1 && tail -1 gpurun_out/bench_final.log > gpurun_out/bench_final.json && cut -c1-600 gpurun_out/bench_final.json &&
bash scripts/prof.sh r1h && python scripts/kshape.py $(find gpurun_out/prof_r1h -name "*kernel_trace.csv" | head -1) 7 60 > gpurun_out/shapes_r1h.txt && head -5 gpurun_out/shapes_r1h.txt && grep ROOFLINE gpurun_out/shapes_r1h.txt
