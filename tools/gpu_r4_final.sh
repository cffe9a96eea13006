# Round-4 end-of-session call: every -m gpu test and smoke(), the PMC passes
# at HEAD (instruction mix, waits, LDS, HBM FETCH/WRITE -> pmc_traffic.json),
# the full default bench line with that traffic, rocprofv3 kernel stats of a
# short bench, and the drop-in single-frame timeline.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r4final}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/${tag}_smoke.log 2>&1
bash tools/gpu_r3_bench.sh ${tag}
timeout -k 10 400 bash tools/gpu_r4_dropin.sh ${tag} > gpurun_out/${tag}_dropin.log 2>&1
echo FINALDONE
