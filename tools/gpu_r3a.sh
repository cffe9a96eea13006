# Round-3 check: the whole -m gpu suite, then the default bench line.  A plain
# test failure (pytest rc 1) still runs the bench; anything else (fault, abort,
# timeout) ends the call.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r3a}
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 500 python3 -u bench.py > gpurun_out/${tag}_bench.log 2>&1
echo ALLDONE pytest_rc=$rc
