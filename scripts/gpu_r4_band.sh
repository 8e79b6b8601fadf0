# band weight-gradient variants: alone (A/B), beside the data gradient, and in the step
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/band
o=gpurun_out/band
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "conv_wgrad_halo" > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
for ab in 16=0/1 16=0/2; do
  timeout -k 10 300 python -u scripts/conv_bench.py --abw $ab --only dec > $o/abw.log 2>&1 || { tail $o/abw.log; exit 1; }; cat $o/abw.log
  timeout -k 10 300 python -u scripts/conv_bench.py --abw $ab --only enc > $o/abw.log 2>&1 || { tail $o/abw.log; exit 1; }; cat $o/abw.log
  timeout -k 10 300 python -u scripts/conv_bench.py --abw $ab --only "postnet 512" > $o/abw.log 2>&1 || { tail $o/abw.log; exit 1; }; cat $o/abw.log
done
for v in 0 1 2; do
  FS2_TUNE=16=$v timeout -k 10 300 python -u scripts/conv_bench.py --only dec > $o/pair$v.log 2>&1 || { tail $o/pair$v.log; exit 1; }; echo "v=$v"; cat $o/pair$v.log
done
for v in 0 1 2 0; do
  FS2_TUNE=16=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $o/bench$v.log 2>&1 || { tail -20 $o/bench$v.log; exit 1; }
  tail -1 $o/bench$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['classes']; print('v=$v', d['ms_per_step'], 'ms', {k: c[k]['ms_per_step'] for k in ('wgrad_k9','wgrad_k5','wgrad_k1','conv_k9')}, 'fft', d['fft_block']['fwd_ms_per_block'], d['fft_block']['bwd_ms_per_block'], d['fft_block']['frac_valid'])"
done
for v in 0 1 0 1; do FS2_TUNE=17=$v timeout -k 10 100 python -u scripts/attn_bench.py | grep -v amdgpu | sed "s/^/xg=$v /"; done
