# widened attention epilogue stores (permlane16_swap pairs -> dwordx4): attention tests, kernels alone under
# ablib/libfs2hip_base.so (HEAD) and the working build, step A/B (3 rounds)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/attnst
o=gpurun_out/attnst
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
for i in 1 2; do
  for lib in ablib/libfs2hip_base.so ""; do
    FS2HIP_LIB=$lib timeout -k 10 120 python -u scripts/attn_bench.py > $o/a.log 2>&1 || { tail -20 $o/a.log; exit 1; }
    echo "[${lib:-new}] $(grep -E 'decoder|encoder' $o/a.log | tr '\n' ' ')"
  done
done
for round in 1 2; do
  for spec in "base|FS2HIP_LIB=ablib/libfs2hip_base.so" "new|FS2_X=0"; do
    label=${spec%%|*}; envs=${spec#*|}
    env $envs timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-f32 > $o/b.log 2>&1 || { tail -20 $o/b.log; exit 1; }
    tail -1 $o/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['classes']; print('$label', d['ms_per_step'], 'ms', {k: c[k]['ms_per_step'] for k in ('attention_fwd','attention_bwd','linear_k1','conv_k9')}, 'fft', d['fft_block']['fwd_ms_per_block'], d['fft_block']['bwd_ms_per_block'])"
  done
done
