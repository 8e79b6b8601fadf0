#!/bin/bash
# round-5 records in one GPU call: PMC of the band k=9 weight gradient (v2), the tap-register
# k=9 forward and the attention kernels; the N-rank collective-schedule model; step phases /
# host enqueue; then r3_check.sh (GPU tests, smoke, default bench, kernel-trace profile).
#   bash scripts/gpu_r5_final.sh <tag> [records|check|all]
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-r5}; part=${2:-all}
o=gpurun_out/$tag
mkdir -p $o
if [ $part != check ]; then
timeout -k 10 300 bash scripts/pmc_kernel.sh conv_wgrad_band python3 scripts/conv_bench.py --probe wgrad --only "dec w1" > $o/pmc_wgrad_k9.txt 2>&1 || { tail $o/pmc_wgrad_k9.txt; exit 1; }
timeout -k 10 300 bash scripts/pmc_kernel.sh conv_gemm_tapreg python3 scripts/conv_bench.py --probe fwd --only "dec w1" > $o/pmc_conv_k9_fwd.txt 2>&1 || { tail $o/pmc_conv_k9_fwd.txt; exit 1; }
timeout -k 10 300 bash scripts/pmc_kernel.sh attn python3 scripts/attn_bench.py --probe > $o/pmc_attn.txt 2>&1 || { tail $o/pmc_attn.txt; exit 1; }
grep -E "==|->" $o/pmc_wgrad_k9.txt $o/pmc_conv_k9_fwd.txt $o/pmc_attn.txt
timeout -k 10 600 python -u scripts/dp_collective_model.py --steps 20 > $o/dp.log 2>&1 || { tail -20 $o/dp.log; exit 1; }
tail -12 $o/dp.log
timeout -k 10 300 python -u scripts/step_phases.py > $o/phases.log 2>&1 || { tail -20 $o/phases.log; exit 1; }
timeout -k 10 300 python -u scripts/step_phases.py --py >> $o/phases.log 2>&1 || { tail -20 $o/phases.log; exit 1; }
grep -E "C blocks|ms from" $o/phases.log
fi
if [ $part != records ]; then bash scripts/r3_check.sh $tag; fi
