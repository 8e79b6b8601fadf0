# k = 1 projections: timings, stage sweep, PMC of the QKV forward and the w_2 data gradient; clean step trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/k1
o=gpurun_out/k1
timeout -k 10 200 python -u scripts/k1_bench.py > $o/t.log 2>&1 || { tail $o/t.log; exit 1; }; grep -v amdgpu $o/t.log
timeout -k 10 300 python -u scripts/k1_bench.py --stages > $o/st.log 2>&1 || { tail $o/st.log; exit 1; }; grep -v amdgpu $o/st.log
timeout -k 10 300 bash scripts/pmc_kernel.sh conv_gemm_nt_glds python3 scripts/k1_bench.py --probe "dec qkv fwd" > $o/pmc_qkv.txt 2>&1 || { tail $o/pmc_qkv.txt; exit 1; }
timeout -k 10 300 bash scripts/pmc_kernel.sh conv_gemm_nt_glds python3 scripts/k1_bench.py --probe "dec w2 dgrad" > $o/pmc_w2d.txt 2>&1 || { tail $o/pmc_w2d.txt; exit 1; }
grep -E "==|->" $o/pmc_qkv.txt $o/pmc_w2d.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4c -o r4c --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-traffic --no-f32 --no-roofline > gpurun_out/prof_r4c.log 2>&1 || { tail gpurun_out/prof_r4c.log; exit 1; }
tail -1 gpurun_out/prof_r4c.log | cut -c1-200
f=$(ls gpurun_out/prof_r4c/*kernel_trace.csv gpurun_out/prof_r4c/*/*kernel_trace.csv 2>/dev/null | head -1)
python scripts/kshape.py "$f" 22 80 --stats gpurun_out/prof_r4c_stats.csv > gpurun_out/prof_r4c_shapes.txt
head -70 gpurun_out/prof_r4c_shapes.txt
