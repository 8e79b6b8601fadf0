#!/bin/bash
# round 5: BatchNorm tanh on v_exp / v_rcp (norm.hip tanh_fast) against libm tanhf (the
# previous library, FS2HIP_LIB): BN / parity tests, alone, in the step
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/tanh; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "batchnorm or step or postnet or trajectory" > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
for r in 1 2 3; do
for v in new ref; do
  lib=""
  [ $v = ref ] && lib=scratch/abt/libfs2hip_tanhref.so
  FS2HIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-f32 > $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
  tail -1 $o/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['classes']; print('$v', d['ms_per_step'], 'ms')" || true
done; done
