#!/bin/bash
# round 5: split-K partials ordered by a library event (no host stream sync):
# kernel + parity tests, then same-box step A/B against the previous library (FS2HIP_LIB)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/skev; mkdir -p $o
true
true
for r in 1 2 3; do
  for lib in new prev; do
    if [ $lib = prev ]; then export FS2HIP_LIB=$PWD/scratch/abt/libfs2hip_prev.so; else unset FS2HIP_LIB; fi
    timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-f32 --no-traffic > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
    echo "[$lib] $(tail -1 $o/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["fft_block"]["fwd_ms_per_block"], d["fft_block"]["bwd_ms_per_block"])')"
  done
done
