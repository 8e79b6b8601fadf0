# PMC passes over the decoder k=9 weight gradient (+ reduce) and the QKV k=1 weight gradient
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 bash scripts/pmc_kernel.sh wgrad python3 scripts/conv_bench.py --probe wgrad --only "dec w1" > gpurun_out/pmc_wgrad_k9.txt 2>&1 || { tail gpurun_out/pmc_wgrad_k9.txt; exit 1; }
timeout -k 10 300 bash scripts/pmc_kernel.sh wgrad python3 scripts/conv_bench.py --probe wgrad --only "dec qkv" > gpurun_out/pmc_wgrad_k1.txt 2>&1 || { tail gpurun_out/pmc_wgrad_k1.txt; exit 1; }
grep -E "==|->" gpurun_out/pmc_wgrad_k9.txt gpurun_out/pmc_wgrad_k1.txt
