#!/bin/bash
# round-4 iteration script: focused tests, kernel A/B, optionally the full GPU suite and a bench
#   bash scripts/gpu_r4.sh <tag> [tests-k-expr] [abw-spec] [full] [bench]
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=$1; kexpr=${2:-}; abw=${3:-}; full=${4:-}; bench=${5:-}
o=gpurun_out/$tag
mkdir -p $o
if [ -n "$kexpr" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$kexpr" > $o/tests_focus.log 2>&1 || { tail -30 $o/tests_focus.log; exit 1; }
  tail -3 $o/tests_focus.log
fi
if [ -n "$abw" ]; then
  timeout -k 10 300 python -u scripts/conv_bench.py --abw "$abw" > $o/abw.log 2>&1 || { tail -20 $o/abw.log; exit 1; }
  cat $o/abw.log
  timeout -k 10 300 python -u scripts/conv_bench.py > $o/pair.log 2>&1 || { tail -20 $o/pair.log; exit 1; }
  cat $o/pair.log
fi
if [ "$full" = "full" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/tests_full.log 2>&1 || { tail -30 $o/tests_full.log; exit 1; }
  tail -3 $o/tests_full.log
fi
if [ "$bench" = "bench" ]; then
  for i in 1 2; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $o/bench$i.log 2>&1 || { tail -20 $o/bench$i.log; exit 1; }
    tail -1 $o/bench$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], 'ms', d['value'], {k: (v['ms_per_step'], v['frac']) for k, v in d['roofline']['classes'].items()}, 'fft', d['fft_block']['fwd_ms_per_block'], d['fft_block']['bwd_ms_per_block'], d['fft_block']['frac_valid'])"
  done
fi
