# Round-3 HEAD check: every -m gpu test, smoke(), then the full default bench
# line (traffic from the committed PMC file).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r3head}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/${tag}_smoke.log 2>&1
timeout -k 10 600 python3 -u bench.py --traffic-json profiles/pmc_traffic.json > gpurun_out/${tag}_bench.log 2>&1
echo ALLDONE
