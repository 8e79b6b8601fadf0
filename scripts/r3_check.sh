#!/bin/bash
# One GPU call: gpu tests, smoke, default bench, kernel-trace profile of a short bench run.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=${1:-r3}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_gputest.log 2>&1 || { tail -30 gpurun_out/${tag}_gputest.log; exit 1; }
tail -2 gpurun_out/${tag}_gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -3 gpurun_out/${tag}_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
tail -1 gpurun_out/${tag}_bench.log | cut -c1-600
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o ${tag} --output-format csv \
  -- python bench.py --no-cpu-baseline --no-traffic --no-f32 --steps 20 --warmup 5 > gpurun_out/prof_${tag}.log 2>&1 || { tail -20 gpurun_out/prof_${tag}.log; exit 1; }
echo prof ok
