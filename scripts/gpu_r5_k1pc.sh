#!/bin/bash
# round 5: persistent wave-specialised k = 1 GEMM (FS2_TUNE_K1_PC): parity, alone, in the step
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/k1pc; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "k1_persistent or k1_bf16_epilogue" > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -3 $o/t.log
timeout -k 10 300 python -u scripts/k1_bench.py --ab 20=0/1 > $o/ab.log 2>&1 || { tail $o/ab.log; exit 1; }; grep -v amdgpu.ids $o/ab.log
timeout -k 10 300 python -u scripts/k1_bench.py --ab 20=0/2 > $o/ab2.log 2>&1 || { tail $o/ab2.log; exit 1; }; grep -v amdgpu.ids $o/ab2.log
for r in 1 2; do
for v in "" 20=1; do
  FS2_TUNE=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-f32 > $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
  tail -1 $o/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['classes']; print('[$v]', d['ms_per_step'], 'ms', {k: c[k]['ms_per_step'] for k in c}, 'fft', d['fft_block']['fwd_ms_per_block'], d['fft_block']['bwd_ms_per_block'], d['fft_block']['frac_valid'])" || true
done; done
