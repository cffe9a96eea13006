# SearchForInitialization variants: capacity / parity tests, then the headline bench line.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-match}
timeout -k 10 400 python -u -m pytest tests/test_match_capacity.py tests/test_gpu_parity.py tests/test_adapter.py -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1
timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1
echo ALLDONE
