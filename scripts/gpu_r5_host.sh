#!/bin/bash
# round 5: host enqueue profile with the backward on the profiled thread; attention PMC
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/host; mkdir -p $o
timeout -k 10 300 python -u scripts/host_profile.py --one-thread > $o/host1.log 2>&1 || { tail -20 $o/host1.log; exit 1; }
head -100 $o/host1.log
timeout -k 10 300 bash scripts/pmc_kernel.sh attn python3 scripts/attn_bench.py --probe > $o/pmc_attn.txt 2>&1 || { tail $o/pmc_attn.txt; exit 1; }
grep -E "==|->|LDS|MFMA_MOPS|INSTS" $o/pmc_attn.txt
