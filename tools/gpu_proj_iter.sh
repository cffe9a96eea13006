# Projection matcher iteration: parity tests + kernel stats of the proj tests.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_proj.py tests/test_adapter.py > gpurun_out/proj_par.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/proj_ks -o ks -- python3 -m pytest -x -q -m gpu tests/test_proj.py > gpurun_out/proj_ks.log 2>&1
echo ALLDONE
