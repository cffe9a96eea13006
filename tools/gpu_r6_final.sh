# Round-6 final call at HEAD: every -m gpu test and smoke(), the PMC passes
# (instruction mix, waits, LDS, HBM FETCH/WRITE -> pmc_traffic.json), the full
# default bench line with that traffic, rocprofv3 kernel stats + trace of a short
# bench with per-launch median / min / max of pyramid, FAST, octree, describe and
# the 256-keypoint matcher (tools/kernel_launches.py), the stereo drop-in tail
# and the single-frame drop-in timeline.   usage: bash tools/gpu_r6_final.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6final}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/${tag}_smoke.log 2>&1
bash tools/gpu_r3_bench.sh ${tag}
python3 tools/kernel_launches.py gpurun_out/${tag}_ks/ks_kernel_trace.csv --kernel pyramid_tick:512 --kernel fast_cells:417280 \
  --kernel octree_kernel:4096 --kernel describe_kernel:262144 --kernel match_init_kernel:512 --between pyramid_tick:512 \
  --json gpurun_out/${tag}_launches.json > /dev/null 2>&1 || echo "launches failed"
REPS=1000 timeout -k 10 400 bash tools/gpu_r5_stereo.sh ${tag} > gpurun_out/${tag}_stereo.log 2>&1
timeout -k 10 400 bash tools/gpu_r4_dropin.sh ${tag} > gpurun_out/${tag}_dropin.log 2>&1
echo FINALDONE
