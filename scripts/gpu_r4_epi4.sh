# bf16 whole-tile epilogue in conv_gemm_tapreg: kernel tests, k=1 projections alone under ablib (HEAD) and the
# working build, then step A/B (3 rounds)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/epi4
o=gpurun_out/epi4
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
for lib in ablib/libfs2hip_base.so ""; do
  FS2HIP_LIB=$lib timeout -k 10 120 python -u scripts/conv_bench.py --only "dec w1" > $o/ln.log 2>&1 || { tail -20 $o/ln.log; exit 1; }
  echo "lib=[${lib:-new}]"; grep -v amdgpu.ids $o/ln.log
done
for round in 1 2 3; do
  for spec in "base|FS2HIP_LIB=ablib/libfs2hip_base.so" "new|FS2_X=0"; do
    label=${spec%%|*}; envs=${spec#*|}
    env $envs timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-f32 > $o/b.log 2>&1 || { tail -20 $o/b.log; exit 1; }
    tail -1 $o/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['classes']; print('$label', d['ms_per_step'], 'ms', {k: c[k]['ms_per_step'] for k in ('linear_k1','conv_k9','conv_k5','wgrad_k9','wgrad_k5','attention_bwd')}, 'fft', d['fft_block']['fwd_ms_per_block'], d['fft_block']['bwd_ms_per_block'])"
  done
done
