cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for spec in "$@"; do
  timeout -k 10 200 python -u scripts/conv_bench.py --ab $spec --reps 20 --only ${ONLY:-dec} > gpurun_out/ab_${spec////_}.log 2>&1 || { cat gpurun_out/ab_${spec////_}.log; exit 1; }
  echo "== $spec"; grep -v amdgpu.ids gpurun_out/ab_${spec////_}.log
done
for spec in $ABW; do
  timeout -k 10 200 python -u scripts/conv_bench.py --abw $spec --reps 20 --only ${ONLY:-dec} > gpurun_out/abw_${spec////_}.log 2>&1 || { cat gpurun_out/abw_${spec////_}.log; exit 1; }
  echo "== w $spec"; grep -v amdgpu.ids gpurun_out/abw_${spec////_}.log
done
