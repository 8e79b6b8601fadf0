#!/bin/bash
# PMC pass over the fused ResBlock kernels (bench_infer.py, bf16)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rbpmc
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  -d gpurun_out/rbpmc/p1 -o p1 --output-format csv -- python bench_infer.py --iters 2 --warmup 1 > gpurun_out/rbpmc/p1.log 2>&1 || { tail -5 gpurun_out/rbpmc/p1.log; exit 1; }
python - <<'PY'
import csv, glob, collections
for kn in ("resblock1_fused<32", "resblock1_fused<64", "conv_gemm_halo<64, 128, 2, 16, true"):
    acc = collections.defaultdict(list)
    for f in glob.glob("gpurun_out/rbpmc/p1/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kn in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(kn)
    for k, v in sorted(acc.items()):
        print(f"  {k:28s} n={len(v):3d} mean={sum(v)/len(v):.4g}")
PY
