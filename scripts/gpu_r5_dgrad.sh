#!/bin/bash
# round 5: decoder k=9 data-gradient tiles beside the band v2 weight gradient (FS2_TUNE_TAPREG
# 0 = 128x128 @2/CU for c_out <= 256, 1 = 128x64 @3/CU), alone / pair / step; host profile
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/dgrad; mkdir -p $o
for v in "" 15=1; do
  FS2_TUNE=$v timeout -k 10 300 python -u scripts/conv_bench.py --only dec > $o/pair.log 2>&1 || { tail $o/pair.log; exit 1; }; echo "[$v]"; grep -v amdgpu.ids $o/pair.log | head -1
done
for r in 1 2; do
for v in "" 15=1; do
  FS2_TUNE=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-f32 > $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
  tail -1 $o/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['classes']; o=d['fft_block']['ops']; print('[$v]', d['ms_per_step'], 'ms', {k: c[k]['ms_per_step'] for k in c}, 'fft', d['fft_block']['fwd_ms_per_block'], d['fft_block']['bwd_ms_per_block'], d['fft_block']['frac_valid'], 'w1 dgrad', o['bwd:w1_k9_dgrad']['ms_per_block'], 'w1 wgrad', o['bwd:w1_k9_wgrad']['ms_per_block'])" || true
done; done
timeout -k 10 300 python -u scripts/host_profile.py > $o/host.log 2>&1 || { tail -20 $o/host.log; exit 1; }
head -40 $o/host.log
