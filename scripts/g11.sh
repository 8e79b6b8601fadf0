set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo NEW; timeout -k 10 300 python scripts/attn_bench.py
echo OLD; FS2HIP_LIB=$PWD/ablib/libfs2hip_old.so timeout -k 10 300 python scripts/attn_bench.py
echo NEW; timeout -k 10 300 python scripts/attn_bench.py
