#!/bin/bash
# round 5: encoder weight re-layout on the side stream (model.ENC_PREP_SIDE) -- same-box step A/B and
# forward phase
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/enc; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_dp.py tests/test_resume.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
for r in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 200 python -u scripts/bench_ab.py model.ENC_PREP_SIDE=$v -- --steps 30 --warmup 5 --no-cpu-baseline --no-f32 --no-traffic > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
    echo "[ENC_PREP_SIDE=$v] $(tail -1 $o/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
timeout -k 10 300 python -u scripts/step_phases.py > $o/phases.log 2>&1 || { tail -20 $o/phases.log; exit 1; }
grep -E "C blocks|ms from" $o/phases.log
