# same-box: round-1 library (scratch/r1, built from 3e2ba81) vs HEAD (tap-register convs) vs HEAD with
# the round-2 halo kernels (FS2_TUNE 19=-1): k=9 convs alone and with the weight gradient on a side
# stream (scripts/conv_bench.py), then each tree's own bench.py step and kernel trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r1ab
R1=$GRAFT_REPO_ROOT/scratch/r1
for cfg in "r1" "head_r2kernels" "head"; do
  case $cfg in r1) L=$R1/mid-attribute-speaker-generation_amd/csrc/libfs2hip.so; T="";; head_r2kernels) L=""; T="19=-1";; head) L=""; T="";; esac
  FS2HIP_LIB=$L FS2_TUNE=$T timeout -k 10 200 python -u scripts/conv_bench.py --only "dec w1" > gpurun_out/r1ab/cb_$cfg.log 2>&1 || { cat gpurun_out/r1ab/cb_$cfg.log; exit 1; }
  FS2HIP_LIB=$L FS2_TUNE=$T timeout -k 10 200 python -u scripts/conv_bench.py --only "enc w1" >> gpurun_out/r1ab/cb_$cfg.log 2>&1 || { cat gpurun_out/r1ab/cb_$cfg.log; exit 1; }
  echo "[$cfg]"; grep -v amdgpu gpurun_out/r1ab/cb_$cfg.log
done
(cd $R1 && timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-traffic > $GRAFT_REPO_ROOT/gpurun_out/r1ab/bench_r1.log 2>&1) || { tail gpurun_out/r1ab/bench_r1.log; exit 1; }
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-traffic --no-f32 > gpurun_out/r1ab/bench_head.log 2>&1 || exit 1
(cd $R1 && timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-traffic > $GRAFT_REPO_ROOT/gpurun_out/r1ab/bench_r1b.log 2>&1) || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-traffic --no-f32 > gpurun_out/r1ab/bench_head_b.log 2>&1 || exit 1
for f in bench_r1 bench_head bench_r1b bench_head_b; do echo "$f $(tail -1 gpurun_out/r1ab/$f.log | cut -c1-250)"; done
(cd $R1 && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r1ab/tr_r1 -o tr --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-traffic --no-roofline > $GRAFT_REPO_ROOT/gpurun_out/r1ab/tr_r1.log 2>&1) || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r1ab/tr_head -o tr --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-traffic --no-roofline --no-f32 > gpurun_out/r1ab/tr_head.log 2>&1 || exit 1
echo traces ok
