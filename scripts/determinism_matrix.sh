#!/bin/bash
# Repeat-run matrix of tests/stale_probe.py (run under gpurun): plain runs (caching allocator,
# no poison), poisoned runs with the same byte twice and with another byte; every pair compared.
# Tells run-to-run nondeterminism (same byte differs) from stale reads (only bytes differ).
#   bash scripts/determinism_matrix.sh <tag> [probe args...]
set -u
tag=$1; shift
o=gpurun_out/$tag; mkdir -p $o
names=()
run() {
  local n=$1; shift
  timeout -k 10 300 python -u tests/stale_probe.py "$@" --out /tmp/dm_$n.pt > $o/$n.log 2>&1 || { echo "probe $n failed"; tail -5 $o/$n.log; exit 1; }
  names+=($n)
}
run plain1 --poison 0 --plain "$@"
run plain2 --poison 0 --plain "$@"
run plain3 --poison 0 --plain "$@"
run p0a --poison 0 "$@"
run p0b --poison 0 "$@"
run p63 --poison 63 "$@"
for ((i = 0; i < ${#names[@]}; i++)); do
  for ((j = i + 1; j < ${#names[@]}; j++)); do
    a=${names[$i]}; b=${names[$j]}
    r=$(python3 tests/stale_probe.py --compare /tmp/dm_$a.pt /tmp/dm_$b.pt 2>&1 | head -3 | cut -c1-300)
    echo "$a vs $b: $r"
  done
done
