# step-level A/B of env configurations: bash scripts/gpu_r4_step.sh "<label>|<env assignments>" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/step
o=gpurun_out/step
for round in 1 2; do
  for spec in "$@"; do
    label=${spec%%|*}; envs=${spec#*|}
    env $envs timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $o/b.log 2>&1 || { tail -20 $o/b.log; exit 1; }
    tail -1 $o/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['classes']; print('$label', d['ms_per_step'], 'ms', {k: c[k]['ms_per_step'] for k in ('wgrad_k9','wgrad_k5','wgrad_k1','conv_k9','attention_fwd','attention_bwd')}, 'fft', d['fft_block']['fwd_ms_per_block'], d['fft_block']['bwd_ms_per_block'], d['fft_block']['frac_valid'])"
  done
done
