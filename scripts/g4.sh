set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o probe --output-format csv -- python bench.py --probe-conv > gpurun_out/pmc.log 2>&1 || { tail -20 gpurun_out/pmc.log; exit 1; }
find gpurun_out/pmc -name "*.csv" | head; f=$(find gpurun_out/pmc -name "*counter_collection.csv" | head -1); head -3 "$f"
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
