# GPU test subset: bash tools/gpu_tests.sh <tag> <pytest args...>
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu "$@" > gpurun_out/$tag.log 2>&1
echo DONE
