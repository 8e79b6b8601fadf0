# hardware-queue check of the data-parallel step at N = 1 (FS2_DP1=1), three fresh processes, and the plain step
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/q
for run in dp1a dp1b dp1c plain; do
  if [ ${run:0:3} = dp1 ]; then export FS2_DP1=1; else export FS2_DP1=0; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/q/$run -o t --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-f32 --no-traffic --no-roofline > gpurun_out/q/$run.log 2>&1 || { tail gpurun_out/q/$run.log; exit 1; }
  echo "== $run $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/q/$run.log)"
  python3 scripts/queue_check.py $(ls gpurun_out/q/$run/*/t_kernel_trace.csv gpurun_out/q/$run/t_kernel_trace.csv 2>/dev/null | head -1)
done
