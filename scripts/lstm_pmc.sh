#!/bin/bash
# PMC passes over the stacked LSTM step kernels (scripts/lstm_bench.py with LSTM_PROBE=1)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lpmc
export LSTM_PROBE=1
i=0
for ctrs in "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAVES SQ_INSTS_VMEM SQ_WAIT_ANY" \
            "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" "TA_BUSY_avr TA_BUSY_max"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d gpurun_out/lpmc/p$i -o p$i --output-format csv -- python scripts/lstm_bench.py > gpurun_out/lpmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/lpmc/p$i.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
for kn in ("lstm_stack_fwd_step", "lstm_stack_bwd_step"):
    print(kn)
    for f in sorted(glob.glob("gpurun_out/lpmc/p*/**/*counter_collection.csv", recursive=True)):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if kn in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            v = v[10:140]  # steady-state launches (all layers active)
            print(f"  {k:28s} n={len(v):3d} mean={sum(v)/len(v):.4g}")
PY
