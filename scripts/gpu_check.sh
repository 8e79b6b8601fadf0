#!/bin/bash
# GPU-box check: parity tests, smoke, short bench.  Stops at the first crash/timeout
# (test *failures* exit 1 and let the later steps run).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -o faulthandler_timeout=240 \
    ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
src=$?
tail -8 gpurun_out/smoke.log
if [ $src -ne 0 ] && [ $src -ne 1 ]; then echo "smoke rc=$src: stopping"; exit $src; fi
timeout -k 10 420 python bench.py --steps ${BENCH_STEPS:-10} --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
brc=$?
tail -5 gpurun_out/bench.log
exit $(( rc | src | brc ))
