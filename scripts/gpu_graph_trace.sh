cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gtr -o g --output-format csv -- python3 bench.py --graph --steps 5 --warmup 3 --no-cpu-baseline --no-f32 --no-traffic --no-roofline > gpurun_out/gtr.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/etr -o e --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-f32 --no-traffic --no-roofline > gpurun_out/etr.log 2>&1 || exit 1
echo ok
