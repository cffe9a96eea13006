# A/B of pyramid build variants on the GPU box (kernel time of a short bench
# under rocprofv3 for each library).  usage: bash tools/gpu_pyr_ab.sh <tag> <lib>...
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "pyramid or extract_mono" > gpurun_out/${tag}_par.log 2>&1
for lib in "$@"; do
  n=$(basename $lib .so)
  ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "pyramid_levels" > gpurun_out/${tag}_${n}_par.log 2>&1
  ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_${n} -o ks -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${tag}_${n}.log 2>&1
done
echo ALLDONE
