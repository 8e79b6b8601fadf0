#!/bin/bash
# wide-tile weight gradient: parity, alone A/B against the band / halo kernels, step A/B
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/wide; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv_wgrad_halo" > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
for sh in dec enc "postnet 512" "postnet in" "postnet out" "vp k3 T128"; do
  timeout -k 10 300 python -u scripts/conv_bench.py --abw 19=-1/0 --only "$sh" > $o/abw.log 2>&1 || { tail $o/abw.log; exit 1; }; cat $o/abw.log
done
FS2_TUNE=19=0 timeout -k 10 300 python -u scripts/conv_bench.py --only dec > $o/pair.log 2>&1 || { tail $o/pair.log; exit 1; }; cat $o/pair.log
for v in -1 0 -1 0; do
  FS2_TUNE=19=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-f32 > $o/bench$v.log 2>&1 || { tail -20 $o/bench$v.log; exit 1; }
  tail -1 $o/bench$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['classes']; print('v=$v', d['ms_per_step'], 'ms', {k: c[k]['ms_per_step'] for k in ('wgrad_k9','wgrad_k5','wgrad_k3','wgrad_k1','conv_k9')}, 'fft', d['fft_block']['fwd_ms_per_block'], d['fft_block']['bwd_ms_per_block'], d['fft_block']['frac_valid'])"
done
