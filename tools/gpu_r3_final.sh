# Round-3 end-of-session call: every -m gpu test and smoke(), PMC passes at
# HEAD (instruction mix, waits, LDS, HBM FETCH/WRITE -> pmc_traffic.json),
# the full default bench line with that traffic, rocprofv3 kernel stats of a
# short bench, and the drop-in latencies with their per-process kernel stats.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r3final}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/${tag}_smoke.log 2>&1
bash tools/gpu_r3_bench.sh ${tag}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_dk -o dk_%pid% -- python3 tools/dropin_profile.py 10 > gpurun_out/${tag}_dk.log 2>&1
timeout -k 10 300 python3 -u tools/pnp_batch_timing.py > gpurun_out/${tag}_pnpbatch.json 2> gpurun_out/${tag}_pnpbatch.err
echo FINALDONE
