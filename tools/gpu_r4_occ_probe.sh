# FAST occupancy probe: the product library against diagnostic builds with
# a shorter survivor list (less LDS per wave, more waves per CU; results are
# wrong only for cells with more survivors -- the parity log says whether the
# test frames have any) and with extra LDS per wave.  Timing lines only.
# usage: bash tools/gpu_r4_occ_probe.sh <tag> <variant>...
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
L=$GRAFT_REPO_ROOT/orb-slam2-annotation_amd
for v in "$@"; do
  ORBGPU_LIBRARY=$L/liborbgpu_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/${tag}_par_$v.log 2>&1 || echo "variant $v parity rc $?"
done
for rep in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras > gpurun_out/${tag}_base_$rep.log 2>&1
  for v in "$@"; do
    ORBGPU_LIBRARY=$L/liborbgpu_$v.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras > gpurun_out/${tag}_${v}_$rep.log 2>&1
  done
done
echo OCCDONE
