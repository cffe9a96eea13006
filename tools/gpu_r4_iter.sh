# Round-4 kernel iteration: extraction parity (+ extra test files given),
# a bench line without extras / CPU legs, the phase stamps of the diagnostic
# build (liborbgpu_xs.so) and kernel stats of a short bench.
# usage: bash tools/gpu_r4_iter.sh <tag> [test files...]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py "$@" > gpurun_out/${tag}_par.log 2>&1
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras > gpurun_out/${tag}_bench.log 2>&1
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --deliver gpu0 > gpurun_out/${tag}_bench2.log 2>&1
if [ -f orb-slam2-annotation_amd/liborbgpu_xs.so ]; then
  ORBGPU_LIBRARY=orb-slam2-annotation_amd/liborbgpu_xs.so timeout -k 10 200 python3 tools/extract_stamps.py > gpurun_out/${tag}_stamps.json 2>&1 || echo "stamps run failed"
fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_ks -o ks -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${tag}_ks.log 2>&1
echo ITERDONE
