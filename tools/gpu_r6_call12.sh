# Round-6 call 12: the whole -m gpu suite on the default build (single-frame
# completion flag), the single-frame A/B (flag vs hipStreamSynchronize) and the
# drop-in C++ classes' latency with each.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r6o_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/r6o_tests.log; exit $rc; }
tail -2 gpurun_out/r6o_tests.log
ROUNDS=3 bash tools/gpu_r6_single3.sh r6o flag:liborbgpu sync:liborbgpu:ORBGPU_SINGLE_DONE_FLAG=0
for r in 1 2; do
  timeout -k 10 300 python3 -u tools/dropin_probe.py > gpurun_out/r6o_dropin_flag_$r.json 2> gpurun_out/r6o_dropin_flag_$r.err || { echo "dropin flag failed"; exit 3; }
  ORBGPU_SINGLE_DONE_FLAG=0 timeout -k 10 300 python3 -u tools/dropin_probe.py > gpurun_out/r6o_dropin_sync_$r.json 2> gpurun_out/r6o_dropin_sync_$r.err || { echo "dropin sync failed"; exit 3; }
done
echo CALL12DONE
