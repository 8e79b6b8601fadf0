#!/bin/bash
# round 5: band weight gradient v2 against v1 (the round-4 library, FS2HIP_LIB) in the step,
# interleaved on one box
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/bandab; mkdir -p $o
for r in 1 2 3; do
for v in v2 v1 v2m; do
  lib=""; tune=""
  [ $v = v1 ] && lib=scratch/ab/libfs2hip_band1.so
  [ $v = v2m ] && tune=19=-1
  FS2HIP_LIB=$lib FS2_TUNE=$tune timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-f32 > $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
  tail -1 $o/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['classes']; print('$v', d['ms_per_step'], 'ms', {k: c[k]['ms_per_step'] for k in c}, 'fft', d['fft_block']['fwd_ms_per_block'], d['fft_block']['bwd_ms_per_block'], d['fft_block']['frac_valid'])" || true
done; done
