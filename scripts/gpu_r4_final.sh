#!/bin/bash
# round-4 records in one GPU call: PMC of the weight-gradient kernels (band k=9, grouped k=1) and
# the k=9 conv, DP1 vs plain steps (3 runs each, interleaved), step phases / host enqueue, then
# r3_check.sh (GPU tests, smoke, default bench, kernel-trace profile).
#   bash scripts/gpu_r4_final.sh <tag> [records|check|all]
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-r4}; part=${2:-all}
o=gpurun_out/$tag
mkdir -p $o
if [ $part != check ]; then
timeout -k 10 300 bash scripts/pmc_kernel.sh conv_wgrad_band python3 scripts/conv_bench.py --probe wgrad --only "dec w1" > $o/pmc_wgrad_k9.txt 2>&1 || { tail $o/pmc_wgrad_k9.txt; exit 1; }
timeout -k 10 300 bash scripts/pmc_kernel.sh wgrad_k1_multi python3 scripts/k1_multi_bench.py --probe > $o/pmc_wgrad_k1.txt 2>&1 || { tail $o/pmc_wgrad_k1.txt; exit 1; }
timeout -k 10 300 bash scripts/pmc_kernel.sh conv_gemm_tapreg python3 scripts/conv_bench.py --probe fwd --only "dec w1" > $o/pmc_conv_k9_fwd.txt 2>&1 || { tail $o/pmc_conv_k9_fwd.txt; exit 1; }
grep -E "==|->" $o/pmc_wgrad_k9.txt $o/pmc_wgrad_k1.txt $o/pmc_conv_k9_fwd.txt
for i in 1 2 3; do
  for mode in plain dp1; do
    if [ $mode = dp1 ]; then e="FS2_DP1=1"; else e="FS2_DP1=0"; fi
    env $e timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-f32 > $o/$mode$i.log 2>&1 || { tail -20 $o/$mode$i.log; exit 1; }
    echo "$mode $i $(tail -1 $o/$mode$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
timeout -k 10 300 python -u scripts/step_phases.py > $o/phases.log 2>&1 || { tail -20 $o/phases.log; exit 1; }
tail -15 $o/phases.log
fi
if [ $part != records ]; then bash scripts/r3_check.sh $tag; fi
