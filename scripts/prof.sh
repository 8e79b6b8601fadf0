#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run: scripts/prof.sh <tag> [bench args]
set -u
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o $tag --output-format csv \
  -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-traffic "$@" > gpurun_out/prof_$tag.log 2>&1
rc=$?
tail -1 gpurun_out/prof_$tag.log | cut -c1-300
exit $rc
