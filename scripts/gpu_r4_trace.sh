# kernel trace of the step (rocprofv3 --kernel-trace --stats) -> per-shape table
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-r4tr}
bash scripts/prof.sh $tag --steps 20 || exit 1
f=$(ls gpurun_out/prof_$tag/*kernel_trace.csv gpurun_out/prof_$tag/*/*kernel_trace.csv 2>/dev/null | head -1)
python scripts/kshape.py "$f" 25 70 --stats gpurun_out/prof_${tag}_stats.csv > gpurun_out/prof_${tag}_shapes.txt
head -60 gpurun_out/prof_${tag}_shapes.txt
