#!/bin/bash
# LDS bank-conflict survey of one short training-step run: per kernel (name x grid), the share of
# LDS-array cycles that are conflict cycles (one rocprofv3 --pmc pass):  bash scripts/lds_conflicts.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/ldsc
mkdir -p $out
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $out -o ldsc --output-format csv \
  -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --no-f32 --no-roofline > $out/run.log 2>&1 || { echo "pmc pass failed"; tail -5 $out/run.log; exit 1; }
python - "$out" <<'PY'
import csv, glob, collections, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        key = (r["Kernel_Name"][:80], r.get("Grid_Size", r.get("Grid_Size_X", "")))
        acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            cnt[key] += 1
rows = []
for k, d in acc.items():
    a, c = d.get("SQ_LDS_IDX_ACTIVE", 0), d.get("SQ_LDS_BANK_CONFLICT", 0)
    rows.append((d.get("GRBM_GUI_ACTIVE", 0), c / a if a else 0, c, a, cnt[k], k))
rows.sort(reverse=True)
print(f"{'GRBM':>10} {'confl/LDS':>9} {'conflict':>10} {'LDS cyc':>10} {'n':>4}  kernel (grid)")
for g, fr, c, a, n, k in rows[:40]:
    print(f"{g:10.3g} {fr:9.3f} {c:10.3g} {a:10.3g} {n:4d}  {k[0]} ({k[1]})")
PY
