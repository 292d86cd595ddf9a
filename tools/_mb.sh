set -o pipefail
mkdir -p gpurun_out/mb26
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "temporal_attn or groupnorm" --timeout 120 --timeout-method thread > gpurun_out/mb26/pytest.log 2>&1 &&
ACTH_LIB=$PWD/ab/lib_pk.so timeout -k 10 120 python -u tools/bench_attn.py > gpurun_out/mb26/old.log 2>&1 &&
timeout -k 10 120 python -u tools/bench_attn.py > gpurun_out/mb26/new.log 2>&1
