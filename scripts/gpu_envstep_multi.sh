# same-box step A/B over several environment settings, one bench run each per round:
#   bash scripts/gpu_envstep_multi.sh ROUNDS "ENV=a" "ENV=b ENV2=c" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
R=$1; shift
for r in $(seq $R); do
  for t in "$@"; do
    env $t timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-f32 --no-traffic > gpurun_out/envab.log 2>&1 || { tail -20 gpurun_out/envab.log; exit 1; }
    echo "[$t] $(tail -1 gpurun_out/envab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["roofline"]["classes"]; print(d["ms_per_step"], "k9", c["conv_k9"]["ms_per_step"], "wk9", c["wgrad_k9"]["ms_per_step"], "fft", d["fft_block"]["fwd_ms_per_block"], d["fft_block"]["bwd_ms_per_block"])')"
  done
done
