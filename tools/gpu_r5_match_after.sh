# Matcher placement A/B: the bench line (no extras / CPU legs, 40 timed steps
# after 20 warm-up steps) with ORBGPU_MATCH_TINY 0/1 and --match-after
# fast_cells / octree / pyramid, interleaved over $ROUNDS rounds.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
B="python3 -u bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 20"
for r in $(seq 1 ${ROUNDS:-2}); do
  ORBGPU_MATCH_TINY=0 timeout -k 10 200 $B > gpurun_out/${tag}_t0_fast_$r.log 2>&1
  for ma in fast_cells octree pyramid; do
    ORBGPU_MATCH_TINY=1 timeout -k 10 200 $B --match-after $ma > gpurun_out/${tag}_t1_${ma}_$r.log 2>&1
  done
  for k in 2048 2560; do
    ORBGPU_MATCH_TINY=1 ORBGPU_OCT_KCAP_A=$k timeout -k 10 200 $B > gpurun_out/${tag}_t1_kcap${k}_$r.log 2>&1
  done
done
echo MADONE
