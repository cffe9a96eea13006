# Pyramid iteration on the GPU box: parity of the pyramid/extraction path,
# per-tick timeline (stamps build), rocprofv3 kernel stats of a short bench.
# usage: bash tools/gpu_pyr_iter.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-pyr}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/${tag}_par.log 2>&1
ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_stamps.so timeout -k 10 200 python tools/pyr_ticks.py > gpurun_out/${tag}_ticks.log 2>&1 || true
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_ks -o ks -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${tag}_ks.log 2>&1
echo ALLDONE
