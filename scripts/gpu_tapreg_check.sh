cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "tapreg or bf16_halo" > gpurun_out/t2_test.log 2>&1; rc=$?; tail -15 gpurun_out/t2_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/conv_bench.py --ab 19=-1/0 --reps 20 > gpurun_out/t2_ab.log 2>&1; rc=$?; cat gpurun_out/t2_ab.log; exit $rc
