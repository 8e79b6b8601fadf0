#!/bin/bash
# round 5: band weight gradient v2 (fixed-offset fragment reads, lens list in LDS, buffer DMA,
# VGPR-form MFMA: 220 VGPRs) vs the wide kernel v2 (+ one-block-per-CU LDS pad): parity, alone,
# beside the data gradient, in the step, PMC
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/wide3; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv_wgrad_halo" > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
for sh in dec enc "postnet 512"; do
  timeout -k 10 300 python -u scripts/conv_bench.py --abw 19=-1/1 --only "$sh" > $o/abw.log 2>&1 || { tail $o/abw.log; exit 1; }; grep -v amdgpu.ids $o/abw.log | head -1
done
FS2_TUNE=19=1 timeout -k 10 300 python -u scripts/conv_bench.py --abw 20=0/1 --only dec > $o/abw.log 2>&1 || { tail $o/abw.log; exit 1; }; grep -v amdgpu.ids $o/abw.log | head -1
for v in 19=-1 19=1 19=1,20=1; do
  FS2_TUNE=$v timeout -k 10 300 python -u scripts/conv_bench.py --only dec > $o/pair.log 2>&1 || { tail $o/pair.log; exit 1; }; echo "$v"; grep -v amdgpu.ids $o/pair.log | head -1
done
for v in 19=-1 19=1,20=1 19=-1 19=1,20=1; do
  FS2_TUNE=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-f32 > $o/bench.log 2>&1 || { tail -20 $o/bench.log; exit 1; }
  tail -1 $o/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['classes']; print('$v', d['ms_per_step'], 'ms', {k: c[k]['ms_per_step'] for k in c}, 'fft', d['fft_block']['fwd_ms_per_block'], d['fft_block']['bwd_ms_per_block'], d['fft_block']['frac_valid'])" || true
done
timeout -k 10 300 bash scripts/pmc_kernel.sh conv_wgrad_band python3 scripts/conv_bench.py --probe wgrad --only "dec w1" > $o/pmc.txt 2>&1 || { tail $o/pmc.txt; exit 1; }
grep -E "==|->" $o/pmc.txt
