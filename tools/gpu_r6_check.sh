# Round-6 check call: the whole -m gpu suite (not stopping at the first failure)
# and smoke(), then the full default bench line (every leg with its
# parity_vs_oracle object).   usage: bash tools/gpu_r6_check.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6check}
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/${tag}_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/${tag}_smoke.log 2>&1
timeout -k 10 600 python3 -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
echo CHECKDONE
