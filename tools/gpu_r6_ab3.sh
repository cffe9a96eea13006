# Round-6 call 3: VALU issue-cost microbenchmark (the ops FAST / describe use),
# the wave-aggregated octree quadrant histogram (agg): parity, batch and single-frame A/B.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6d}
timeout -k 10 120 tools/valu_rate > gpurun_out/${tag}_valu_rate.txt 2>&1
ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_agg.so timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/${tag}_agg_parity.log 2>&1
NO_PMC=1 ROUNDS=2 bash tools/gpu_r6_libab.sh ${tag} liborbgpu liborbgpu_agg
ROUNDS=3 bash tools/gpu_r6_single.sh ${tag} liborbgpu liborbgpu_agg
echo AB3DONE
