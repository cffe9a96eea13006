# SearchForInitialization block size in the stream bench: the matcher's
# parity tests (every block size, the level-0 bound), then alternated
# default-line benches (no CPU legs, no extras) per ORBGPU_MATCH_THREADS value,
# and the same with the step split in two sub-batches.
# usage: bash tools/gpu_r4_match_ab.sh <tag> <threads>...
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_match_capacity.py \
  tests/test_gpu_parity.py -k "match or init or capacity or block" > gpurun_out/${tag}_par.log 2>&1
for rep in 1 2; do
  for v in "$@"; do
    ORBGPU_MATCH_THREADS=$v timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras > gpurun_out/${tag}_t${v}_$rep.log 2>&1
    ORBGPU_MATCH_THREADS=$v timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --parts 2 --part-stage fast_cells > gpurun_out/${tag}_t${v}_p2_$rep.log 2>&1
  done
done
echo MATCHABDONE
