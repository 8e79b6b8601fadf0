#!/bin/bash
# round 5: FFT blocks from C (bitwise vs the per-kernel path), host enqueue A/B, the stand-in
# collective tests and the N=8 schedule model
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5c; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dp.py -m gpu -x -v --timeout 180 --timeout-method thread -k "c_blocks or fused_gemm_ln or collective_model or bitwise or graph_replay" > $o/t.log 2>&1 || { tail -40 $o/t.log; exit 1; }
grep -E "PASS|FAIL|SKIP|passed|failed" $o/t.log | tail -15
for m in "" --py "" --py; do
  timeout -k 10 300 python -u scripts/step_phases.py $m > $o/phases.log 2>&1 || { tail -20 $o/phases.log; exit 1; }
  tail -3 $o/phases.log
done
timeout -k 10 600 python -u scripts/dp_collective_model.py --ranks 8 --busbw 150,300,450 --steps 20 --rounds 2 > $o/dp.log 2>&1 || { tail -20 $o/dp.log; exit 1; }
cat $o/dp.log
for m in "" --per-kernel-issue "" --per-kernel-issue; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-f32 $m > $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
  tail -1 $o/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['classes']; print('$m', d['ms_per_step'], 'ms', {k: c[k]['ms_per_step'] for k in c}, 'fft', d['fft_block']['fwd_ms_per_block'], d['fft_block']['bwd_ms_per_block'], d['fft_block']['frac_valid'], d['roofline']['kernel'][:60], d['roofline']['frac'])" || true
done
