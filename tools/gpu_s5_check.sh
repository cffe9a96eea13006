set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/s5_gputests.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/s5_bench.log 2>&1
echo ALLDONE
