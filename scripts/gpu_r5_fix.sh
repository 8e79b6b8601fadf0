#!/bin/bash
# round 5: split fixup of the grouped k = 1 weight gradient inside the kernel (last-arriving block
# per tile) vs the separate reduce launch: kernel / parity tests, then same-box step A/B
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/fix; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "k1_multi or blocks or parity or step" > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
for r in 1 2 3; do
  for t in "FS2_TUNE=20=0" "FS2_TUNE=20=1"; do
    env $t timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-f32 --no-traffic > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
    echo "[$t] $(tail -1 $o/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
