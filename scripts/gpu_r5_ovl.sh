#!/bin/bash
# round 5: Adam of the late parameters on the side stream under the next step's encoder forward
# (optimizer.OVERLAP_UPDATE): parity tests, then same-box A/B in the step
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/ovl; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_dp.py tests/test_resume.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
timeout -k 10 300 python -u scripts/step_phases.py > $o/phases.log 2>&1 || { tail -20 $o/phases.log; exit 1; }
grep -E "C blocks|ms from" $o/phases.log
for r in 1 2 3; do
for v in 1 0; do
  timeout -k 10 300 python -u scripts/bench_ab.py optimizer.OVERLAP_UPDATE=$v -- --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-f32 > $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
  tail -1 $o/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('OVERLAP_UPDATE=$v', d['ms_per_step'], 'ms')" || true
done; done
