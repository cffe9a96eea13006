# Round-5 HEAD check: the whole -m gpu suite and smoke(), then the bench line
# (no extras / CPU legs, 40 timed steps after 20 warm-up steps) with each
# delivery mode, interleaved over $ROUNDS rounds, then a kernel trace + stats
# of a short default bench (per-launch durations: tools/pyr_launches.py).
# usage: ROUNDS=2 bash tools/gpu_r5_check.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/${tag}_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/${tag}_smoke.log 2>&1
B="python3 -u bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 20"
for r in $(seq 1 ${ROUNDS:-2}); do
  for d in ${DELIVER_VALS:-gpu0 host}; do
    timeout -k 10 200 $B --deliver $d > gpurun_out/${tag}_deliver_${d}_$r.log 2>&1
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_ks -o ks -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${tag}_ks.log 2>&1
echo CHECKDONE
