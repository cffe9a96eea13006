# Quick check: extractor parity + headline bench line (stage times).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-q}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1
timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1
echo QUICKDONE
