#!/bin/bash
# round-5 baseline on this round's box: default bench (no cpu/f32/traffic legs), the k>=3 convs
# alone and paired (decoder / encoder / PostNet), step phases
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5base; mkdir -p $o
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-f32 > $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
tail -1 $o/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['classes']; print(d['ms_per_step'], 'ms', {k: c[k]['ms_per_step'] for k in c}, 'fft', d['fft_block']['fwd_ms_per_block'], d['fft_block']['bwd_ms_per_block'], d['fft_block']['frac_valid'])"
timeout -k 10 300 python -u scripts/conv_bench.py > $o/conv.log 2>&1 || { tail $o/conv.log; exit 1; }
cat $o/conv.log
timeout -k 10 300 python -u scripts/step_phases.py > $o/phases.log 2>&1 || { tail -20 $o/phases.log; exit 1; }
tail -15 $o/phases.log
