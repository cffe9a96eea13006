# Round-3 check: the whole -m gpu suite, then the default bench line.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r3a}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1
timeout -k 10 500 python3 -u bench.py > gpurun_out/${tag}_bench.log 2>&1
echo ALLDONE
