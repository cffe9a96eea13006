# Round-6 call 19: device-scope ordering events in the bench's stream pipeline
# (orbgpu.DeviceEvent) and no system fence on the extractor's timing events: the
# whole -m gpu suite, the A/B (BENCH_DEVICE_EVENTS 1 vs 0) and one full default line.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r6x_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/r6x_tests.log; exit $rc; }
tail -1 gpurun_out/r6x_tests.log
ROUNDS=3 bash tools/gpu_r6_envab.sh r6x dev sys=BENCH_DEVICE_EVENTS=0
timeout -k 10 600 python3 -u bench.py > gpurun_out/r6x_bench.log 2>&1
tail -c 300 gpurun_out/r6x_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6x_ks -o ks -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/r6x_ks.log 2>&1
echo CALL19DONE
