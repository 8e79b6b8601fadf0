# round-3 final: k9 PMC passes (forward, data gradient), then tests + smoke + bench + kernel trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 bash scripts/pmc_kernel.sh conv_gemm_tapreg python3 scripts/conv_bench.py --probe fwd --only "dec w1" > gpurun_out/fin_pmc_fwd.txt 2>&1 || { tail gpurun_out/fin_pmc_fwd.txt; exit 1; }
timeout -k 10 300 bash scripts/pmc_kernel.sh conv_gemm_tapreg python3 scripts/conv_bench.py --probe dgrad --only "dec w1" > gpurun_out/fin_pmc_dgrad.txt 2>&1 || { tail gpurun_out/fin_pmc_dgrad.txt; exit 1; }
grep -- "->" gpurun_out/fin_pmc_fwd.txt gpurun_out/fin_pmc_dgrad.txt
bash scripts/r3_check.sh r3d
