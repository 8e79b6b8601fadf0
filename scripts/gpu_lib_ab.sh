# conv_bench --ab under two libraries (HEAD build vs $ALT), with and without lens
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for nl in "" 1; do
  for lib in "" "$ALT"; do
    NOLENS=$nl FS2HIP_LIB=$lib timeout -k 10 200 python -u scripts/conv_bench.py --ab ${SPEC:-19=0/0} --reps 20 --only "${ONLY:-dec w1}" > gpurun_out/libab.log 2>&1 || { cat gpurun_out/libab.log; exit 1; }
    echo "nolens=[$nl] lib=[${lib:-HEAD}] $(grep -v amdgpu.ids gpurun_out/libab.log)"
  done
done
