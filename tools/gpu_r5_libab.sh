# Round-5 library A/B: the bench line (no extras / CPU legs, 40 timed steps
# after 20 warm-up steps) for each library named, interleaved over $ROUNDS rounds.
# usage: ROUNDS=2 bash tools/gpu_r5_libab.sh <tag> lib1 lib2 ...   (names without .so)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 20 > gpurun_out/${tag}_${lib}_$r.log 2>&1 || echo "$lib failed"
  done
done
echo LIBABDONE
