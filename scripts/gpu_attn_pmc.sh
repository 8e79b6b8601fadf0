# PMC passes over the decoder-shaped attention kernels (forward, dQ + delta, dK/dV)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 bash scripts/pmc_kernel.sh attn python3 scripts/attn_bench.py --probe > gpurun_out/pmc_attn.txt 2>&1 || { tail gpurun_out/pmc_attn.txt; exit 1; }
grep -E "==|->" gpurun_out/pmc_attn.txt
