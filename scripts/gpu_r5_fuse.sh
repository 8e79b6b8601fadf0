#!/bin/bash
# round 5: post-LN fusions on the encoder too (model.FUSE_LN_MIN_ROWS 4096 vs 16384) -- same-box step A/B and
# forward phase
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/fuse; mkdir -p $o
true
true
for r in 1 2 3; do
  for v in 4096 16384; do
    timeout -k 10 200 python -u scripts/bench_ab.py model.FUSE_LN_MIN_ROWS=$v -- --steps 30 --warmup 5 --no-cpu-baseline --no-f32 --no-traffic > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
    echo "[FUSE_LN_MIN_ROWS=$v] $(tail -1 $o/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
timeout -k 10 300 python -u scripts/step_phases.py > $o/phases.log 2>&1 || { tail -20 $o/phases.log; exit 1; }
grep -E "C blocks|ms from" $o/phases.log
