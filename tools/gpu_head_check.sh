set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/h_gpu_all.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/h_bench.log 2>&1
echo ALLDONE
