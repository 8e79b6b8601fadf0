#!/bin/bash
# PMC passes (one rocprofv3 --pmc run each) over a probe command, averaged per dispatch of the
# kernels whose name contains $1:   bash scripts/pmc_kernel.sh '<name part>' <cmd...>
set -u
pat="$1"; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_$(date +%s)
mkdir -p $out
i=0
for ctrs in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" \
            "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d $out/p$i -o p$i --output-format csv -- "$@" > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
done
python - "$pat" "$out" <<'PY'
import csv, glob, collections, sys
pat, out = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            acc[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for kn, d in acc.items():
    print("==", kn)
    for k, v in sorted(d.items()):
        print(f"   {k:32s} n={len(v):3d} mean={sum(v)/len(v):.4g}")
    g = d.get("GRBM_GUI_ACTIVE"); w = d.get("SQ_WAVE_CYCLES")
    if g and w and d.get("SQ_WAIT_ANY"):
        W = sum(w) / len(w)
        print(f"   -> wait_any {sum(d['SQ_WAIT_ANY'])/len(d['SQ_WAIT_ANY'])/W:.2f}, wait_inst {sum(d['SQ_WAIT_INST_ANY'])/len(d['SQ_WAIT_INST_ANY'])/W:.2f}, active {sum(d['SQ_ACTIVE_INST_ANY'])/len(d['SQ_ACTIVE_INST_ANY'])/W:.2f} of wave cycles")
    if g and d.get("SQ_VALU_MFMA_BUSY_CYCLES"):
        G = sum(g) / len(g)
        print(f"   -> MFMA busy {sum(d['SQ_VALU_MFMA_BUSY_CYCLES'])/len(d['SQ_VALU_MFMA_BUSY_CYCLES'])/(1024*G/8):.3f} (of 1024 SIMDs x GRBM/8), kernel {G/8/2.4e3:.1f} us at 2.4 GHz (GRBM summed over 8 XCDs)")
    if d.get("FETCH_SIZE") and d.get("WRITE_SIZE"):
        print(f"   -> HBM-side bytes: fetch x2 {2*sum(d['FETCH_SIZE'])/len(d['FETCH_SIZE'])/1024:.1f} MB, write {sum(d['WRITE_SIZE'])/len(d['WRITE_SIZE'])/1024:.1f} MB")
PY
