#!/bin/bash
# round 5: mel head / variance predictors issued from C (bitwise tests, host enqueue), band
# weight gradient v2 at 77 KB (two blocks per CU) against v1 in the step (per-kernel issue:
# the round-4 library lacks the new entry points)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/head; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "c_blocks or conv_wgrad_halo or step_bitwise" > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
timeout -k 10 300 python -u scripts/step_phases.py > $o/phases.log 2>&1 || { tail -20 $o/phases.log; exit 1; }
grep -E "C blocks" $o/phases.log
for r in 1 2 3; do
for v in v2 v1; do
  lib=""
  [ $v = v1 ] && lib=scratch/ab/libfs2hip_band1.so
  FS2HIP_LIB=$lib timeout -k 10 300 python -u bench.py --per-kernel-issue --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-f32 > $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
  tail -1 $o/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['classes']; print('$v', d['ms_per_step'], 'ms', {k: c[k]['ms_per_step'] for k in c}, 'fft', d['fft_block']['fwd_ms_per_block'], d['fft_block']['bwd_ms_per_block'], d['fft_block']['frac_valid'])" || true
done; done
