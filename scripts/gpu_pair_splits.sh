# dgrad||wgrad pair of the decoder k=9 conv under weight-gradient split counts (grid sizes)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for t in "" "3=2" "3=4" "3=6" "3=12"; do
  FS2_TUNE=$t timeout -k 10 200 python -u scripts/conv_bench.py --only "${ONLY:-dec w1}" > gpurun_out/pair.log 2>&1 || { cat gpurun_out/pair.log; exit 1; }
  echo "[$t] $(grep -v amdgpu gpurun_out/pair.log | head -1)"
done
