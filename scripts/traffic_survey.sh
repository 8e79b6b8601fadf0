#!/bin/bash
# Per-kernel HBM-side traffic of one short training-step run (two rocprofv3 --pmc passes:
# FETCH_SIZE, WRITE_SIZE; gfx950 correction: FETCH_SIZE x 2 per MI355X_MICROARCH.md), with the
# kernel-trace durations: MB per launch and GB/s, largest first.  bash scripts/traffic_survey.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/traffic
mkdir -p $out
cmd="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --no-f32 --no-roofline"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $out/f -o f --output-format csv -- $cmd > $out/f.log 2>&1 || { echo "fetch pass failed"; tail -3 $out/f.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $out/w -o w --output-format csv -- $cmd > $out/w.log 2>&1 || { echo "write pass failed"; tail -3 $out/w.log; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace -d $out/t -o t --output-format csv -- $cmd > $out/t.log 2>&1 || { echo "trace pass failed"; exit 1; }
python - "$out" <<'PY'
import csv, glob, collections, sys
o = sys.argv[1]
def load(pat, field):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{o}/{pat}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[(r["Kernel_Name"][:70], r.get("Grid_Size", ""))].append(float(r["Counter_Value"]))
    return acc
fe, wr = load("f", "FETCH_SIZE"), load("w", "WRITE_SIZE")
dur = collections.defaultdict(list)
for f in glob.glob(f"{o}/t/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[(r["Kernel_Name"][:70], r.get("Grid_Size", ""))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
rows = []
for k in fe:
    F = 2 * sum(fe[k]) / len(fe[k]) / 1024  # KB -> MB (x2 gfx950)
    W = (sum(wr[k]) / len(wr[k]) / 1024) if k in wr else 0.0
    d = sorted(dur.get(k, [0]))[len(dur.get(k, [0])) // 2] / 1e3
    n = len(fe[k])
    rows.append((n * d, F, W, d, n, k))
rows.sort(reverse=True)
print(f"{'us/run':>8} {'fetch MB':>9} {'write MB':>9} {'us':>7} {'GB/s':>7} {'n':>3}  kernel (grid)")
for tot, F, W, d, n, k in rows[:45]:
    print(f"{tot:8.0f} {F:9.1f} {W:9.1f} {d:7.1f} {(F + W) / d * 1e3 if d else 0:7.0f} {n:3d}  {k[0]} ({k[1]})")
PY
