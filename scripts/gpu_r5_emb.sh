#!/bin/bash
# round 5: embedding scatter-add with 8 ids per block:
# kernel + parity tests, then same-box step A/B against the previous library (FS2HIP_LIB)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/emb; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "embed or bucket or rowvec or index or blocks or parity or step or length" > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
for r in 1 2 3; do
  for lib in new prev; do
    if [ $lib = prev ]; then export FS2HIP_LIB=$PWD/scratch/abt/libfs2hip_prev.so; else unset FS2HIP_LIB; fi
    timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-f32 --no-traffic > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
    echo "[$lib] $(tail -1 $o/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["fft_block"]["fwd_ms_per_block"], d["fft_block"]["bwd_ms_per_block"])')"
  done
done
