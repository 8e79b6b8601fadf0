#!/bin/bash
# round 5: 8-wave 256 x 128 tap-register tiles with deeper weight rings (FS2_TUNE_TAPREG 5: 4
# slots = two tiles in flight, 6: 3 slots) against the default 128 x 64 / 128 x 128 tiles
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/tr8b; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tapreg" > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
for sh in dec "postnet 512"; do
  timeout -k 10 300 python -u scripts/conv_bench.py --ab 15=0/5 --only "$sh" > $o/ab.log 2>&1 || { tail $o/ab.log; exit 1; }; grep -v amdgpu.ids $o/ab.log | head -1
  timeout -k 10 300 python -u scripts/conv_bench.py --ab 15=0/6 --only "$sh" > $o/ab.log 2>&1 || { tail $o/ab.log; exit 1; }; grep -v amdgpu.ids $o/ab.log | head -1
done
