# tapreg: kernel tests, PMC passes on the decoder k=9 fwd / dgrad probes, default bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "tapreg or bf16_halo or conv_gemm" > gpurun_out/r3b_test.log 2>&1 || { tail -30 gpurun_out/r3b_test.log; exit 1; }
tail -1 gpurun_out/r3b_test.log
timeout -k 10 300 bash scripts/pmc_kernel.sh conv_gemm_tapreg python3 scripts/conv_bench.py --probe fwd --only dec > gpurun_out/r3b_pmc_fwd.txt 2>&1 || { tail gpurun_out/r3b_pmc_fwd.txt; exit 1; }
timeout -k 10 300 bash scripts/pmc_kernel.sh conv_gemm_tapreg python3 scripts/conv_bench.py --probe dgrad --only dec > gpurun_out/r3b_pmc_dgrad.txt 2>&1 || { tail gpurun_out/r3b_pmc_dgrad.txt; exit 1; }
grep -- "->" gpurun_out/r3b_pmc_fwd.txt gpurun_out/r3b_pmc_dgrad.txt
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-f32 > gpurun_out/r3b_bench.log 2>&1 || { tail -20 gpurun_out/r3b_bench.log; exit 1; }
tail -1 gpurun_out/r3b_bench.log | cut -c1-400
