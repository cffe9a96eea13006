# Round-5 HEAD check + LDS-DMA A/B: the whole -m gpu suite, then the bench line
# (no extras / CPU legs, 40 timed steps after 20 warm-up steps) with the
# register-staged kernels and with each LDS-DMA width of FAST and describe,
# interleaved over $ROUNDS rounds.
# usage: ROUNDS=2 bash tools/gpu_r5_dma.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/${tag}_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; [ $rc -eq 1 ] || exit $rc; }
B="python3 -u bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 20"
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 200 $B > gpurun_out/${tag}_base_$r.log 2>&1
  for v in ${FAST_VALS:-1 3 8}; do
    ORBGPU_FAST_DMA=$v timeout -k 10 200 $B > gpurun_out/${tag}_fdma${v}_$r.log 2>&1
  done
  for v in ${DESC_VALS:-1 4 16}; do
    ORBGPU_DESC_DMA=$v timeout -k 10 200 $B > gpurun_out/${tag}_ddma${v}_$r.log 2>&1
  done
done
echo DMADONE
