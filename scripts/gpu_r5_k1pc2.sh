#!/bin/bash
# round 5: persistent k = 1 GEMM, second build (tile coordinates decoded once): parity, alone, PMC
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/k1pc2; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "k1_persistent" > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
timeout -k 10 300 python -u scripts/k1_bench.py --ab 20=0/1 > $o/ab.log 2>&1 || { tail $o/ab.log; exit 1; }; grep -v amdgpu.ids $o/ab.log
FS2_TUNE=20=1 timeout -k 10 300 bash scripts/pmc_kernel.sh gemm_k1_pc python3 scripts/k1_bench.py --probe "dec qkv fwd" > $o/pmc.txt 2>&1 || { tail $o/pmc.txt; exit 1; }
grep -E "==|->|LDS|MFMA_MOPS|INSTS" $o/pmc.txt
timeout -k 10 300 bash scripts/pmc_kernel.sh conv_gemm_nt_glds python3 scripts/k1_bench.py --probe "dec qkv fwd" > $o/pmc0.txt 2>&1 || { tail $o/pmc0.txt; exit 1; }
grep -E "==|->|LDS|MFMA_MOPS|INSTS" $o/pmc0.txt
