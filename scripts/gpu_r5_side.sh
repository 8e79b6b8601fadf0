#!/bin/bash
# round 5: embedding-table gradients (bucket / speaker / word / accent) on the side stream, no
# join at the end of the encoder backward: GPU parity / DP / resume tests, then same-box A/B
# against the previous commit's tree (scratch/abt/prev: its host code and its library)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/side; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dp.py tests/test_resume.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not tapreg and not halo" > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
timeout -k 10 300 python -u scripts/step_phases.py > $o/phases.log 2>&1 || { tail -20 $o/phases.log; exit 1; }
grep -E "C blocks|ms from" $o/phases.log
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-f32 > $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
  tail -1 $o/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('side', d['ms_per_step'], 'ms')" || true
  (cd scratch/abt/prev && timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-f32) > $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
  tail -1 $o/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('prev', d['ms_per_step'], 'ms')" || true
done
