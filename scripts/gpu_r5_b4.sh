#!/bin/bash
# round 5: band weight gradient v2 for the taps 3 / 5, 64-multiple-channel convs too
# (FS2_TUNE_WGRAD_BAND 4: PostNet 512 k=5, variance predictors k=3) against the split-K halo
# kernel; C-path bitwise tests and host enqueue after the size-query memo
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/b4; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "c_blocks or step_bitwise" > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
timeout -k 10 300 python -u scripts/step_phases.py > $o/phases.log 2>&1 || { tail -20 $o/phases.log; exit 1; }
grep -E "C blocks|ms from" $o/phases.log
for sh in "postnet 512" "vp k3 T128" "vp k3 T512"; do
  timeout -k 10 300 python -u scripts/conv_bench.py --abw 16=0/4 --only "$sh" > $o/abw.log 2>&1 || { tail $o/abw.log; exit 1; }; grep -v amdgpu.ids $o/abw.log | head -1
done
for r in 1 2 3; do
for v in "" 16=4; do
  FS2_TUNE=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-f32 > $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
  tail -1 $o/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['classes']; print('[$v]', d['ms_per_step'], 'ms', {k: c[k]['ms_per_step'] for k in c}, 'fft', d['fft_block']['fwd_ms_per_block'], d['fft_block']['bwd_ms_per_block'], d['fft_block']['frac_valid'])" || true
done; done
