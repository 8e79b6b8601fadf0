#!/bin/bash
# round 5: 8-wave 256 x 128 tap-register conv tiles (FS2_TUNE_TAPREG 5) against the default
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/tr8; mkdir -p $o
for sh in dec "postnet 512"; do
  timeout -k 10 300 python -u scripts/conv_bench.py --ab 15=0/5 --only "$sh" > $o/ab.log 2>&1 || { tail $o/ab.log; exit 1; }; grep -v amdgpu.ids $o/ab.log
done
for r in 1 2; do
for v in "" 15=5; do
  FS2_TUNE=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-f32 > $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
  tail -1 $o/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['classes']; print('[$v]', d['ms_per_step'], 'ms', {k: c[k]['ms_per_step'] for k in c}, 'fft', d['fft_block']['fwd_ms_per_block'], d['fft_block']['bwd_ms_per_block'], d['fft_block']['frac_valid'])" || true
done; done
