# kernel trace of the N=1 step through the one-rank RCCL data-parallel path (FS2_DP1=1)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
FS2_DP1=1 GPU_MAX_HW_QUEUES=${HWQ:-4} timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/dp1tr -o d --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-f32 --no-traffic --no-roofline > gpurun_out/dp1tr.log 2>&1 || { tail gpurun_out/dp1tr.log; exit 1; }
echo ok
