#!/bin/bash
# The one launcher for GPU-box work (run it under gpurun from the repo root).  Every GPU step
# has its own time limit and the first failure ends the call.
#
#   bash scripts/gpu.sh tests [pytest args]          GPU tests (-m gpu)
#   bash scripts/gpu.sh check <tag>                  tests + smoke + default bench + kernel-trace
#                                                    profile of a short bench run
#   bash scripts/gpu.sh bench <tag> [bench args]     one bench.py line
#   bash scripts/gpu.sh ab <tag> <rounds> <envA> <envB> [<envC> ...] [-- bench args]
#                                                    interleaved same-box bench A/B of environment
#                                                    settings, e.g. "FS2_TUNE=19=-1" or "-" (none)
#   bash scripts/gpu.sh profile <tag> [bench args]   rocprofv3 --kernel-trace --stats of bench.py
#   bash scripts/gpu.sh pmc <tag> <kernel part> <cmd...>
#                                                    PMC passes of one probe command (pmc_kernel.sh)
#   bash scripts/gpu.sh stale                        stale-read probe (tests/stale_probe.py), two
#                                                    poison bytes per path, compared
# Logs and summaries land in gpurun_out/<tag>/.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
cmd=${1:-tests}; shift || true
fail() { echo "FAILED: $1"; tail -30 "$2"; exit 1; }

case $cmd in
tests)
  mkdir -p gpurun_out
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "$@" \
    > gpurun_out/tests.log 2>&1 || fail tests gpurun_out/tests.log
  tail -3 gpurun_out/tests.log ;;
check)
  tag=${1:-check}; o=gpurun_out/$tag; mkdir -p $o
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > $o/tests.log 2>&1 || fail tests $o/tests.log
  tail -2 $o/tests.log
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || fail smoke $o/smoke.log
  tail -3 $o/smoke.log
  timeout -k 10 400 python -u bench.py > $o/bench.log 2>&1 || fail bench $o/bench.log
  tail -1 $o/bench.log | cut -c1-700
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $o/prof -o $tag --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-traffic --no-f32 --steps 20 --warmup 5 \
    > $o/prof.log 2>&1 || fail profile $o/prof.log
  echo profile ok ;;
bench)
  tag=${1:-bench}; shift || true; o=gpurun_out/$tag; mkdir -p $o
  timeout -k 10 600 python -u bench.py "$@" > $o/bench.log 2>&1 || fail bench $o/bench.log
  tail -1 $o/bench.log | cut -c1-1500 ;;
ab)
  tag=$1; rounds=$2; shift 2
  envs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
  [ $# -gt 0 ] && shift
  o=gpurun_out/$tag; mkdir -p $o
  for r in $(seq $rounds); do
    for e in "${envs[@]}"; do
      if [ "$e" = "-" ]; then set_env=(); else set_env=($e); fi
      env "${set_env[@]}" timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline \
        --no-traffic --no-f32 "$@" > $o/ab.log 2>&1 || fail "ab $e" $o/ab.log
      tail -1 $o/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); f=d.get('fft_block',{}); print('$e', d['ms_per_step'], 'ms', 'fft', f.get('fwd_ms_per_block'), f.get('bwd_ms_per_block'), f.get('frac_valid'))"
    done
  done ;;
profile)
  tag=${1:-prof}; shift || true; o=gpurun_out/$tag; mkdir -p $o
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $o/prof -o $tag --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-traffic --no-f32 --steps 20 --warmup 5 "$@" \
    > $o/prof.log 2>&1 || fail profile $o/prof.log
  tail -1 $o/prof.log | cut -c1-400
  python3 scripts/kstats.py "$(find $o/prof -name '*kernel_stats.csv' | head -1)" 25 30 || true ;;
pmc)
  tag=$1; part=$2; shift 2; o=gpurun_out/$tag; mkdir -p $o
  timeout -k 10 600 bash scripts/pmc_kernel.sh "$part" "$@" > $o/pmc.txt 2>&1 || fail pmc $o/pmc.txt
  grep -E "==|->" $o/pmc.txt ;;
stale)
  o=gpurun_out/stale; mkdir -p $o
  run() {  # name, probe args...
    local n=$1; shift
    timeout -k 10 300 python -u tests/stale_probe.py "$@" --out /tmp/stale_$n.pt > $o/$n.log 2>&1
    local rc=$?; tail -2 $o/$n.log; return $rc
  }
  cmp() { python3 tests/stale_probe.py --compare /tmp/stale_$1.pt /tmp/stale_$2.pt > $o/cmp_$1_$2.txt 2>&1; true; }
  run c0 --poison 0 && run c63 --poison 63 && cmp c0 c63 &&
    run k0 --poison 0 --path kernel && run k63 --poison 63 --path kernel && cmp k0 k63 && cmp c0 k0
  rc=$?
  for f in $o/cmp_*.txt; do echo "== $f"; head -40 "$f"; done
  exit $rc ;;
*)
  echo "unknown command $cmd"; exit 2 ;;
esac
