# bench.py eager vs --graph under HIP runtime graph-execution settings (same box)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
run() {  # label, env..., -- bench args
  local label=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-f32 --no-traffic --no-roofline $GARGS > gpurun_out/genv.log 2>&1 || { echo "[$label] FAILED"; tail -5 gpurun_out/genv.log; return 0; }
  echo "[$label] $(tail -1 gpurun_out/genv.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"].get("execution"))')"
}
GARGS="" run eager X=1
GARGS="--graph" run graph X=1
GARGS="--graph" run graph_nocap DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
GARGS="--graph" run graph_q2 DEBUG_HIP_FORCE_GRAPH_QUEUES=2
GARGS="--graph" run graph_nocap_q2 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=2
GARGS="--graph" run graph_nocap_q4 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4
GARGS="" run eager2 X=1
