# Round-6 call 16: the whole -m gpu suite with the relaxed completion-flag store,
# the C++ drop-in extraction latency (1,000 calls x 2) and the single-frame timeline.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r6t_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/r6t_tests.log; exit $rc; }
tail -1 gpurun_out/r6t_tests.log
ROUNDS=2 REPS=1000 timeout -k 10 600 python3 -u tools/extract_cpp_probe.py new > gpurun_out/r6t_cpp.txt 2>&1 || { echo "cpp probe failed"; exit 3; }
cat gpurun_out/r6t_cpp.txt
timeout -k 10 400 bash tools/gpu_r4_dropin.sh r6t > gpurun_out/r6t_dropin.log 2>&1
python3 tools/dropin_timeline.py gpurun_out/r6t_dropin/prof --anchor pyramid_band --before 0 --after 4 > gpurun_out/r6t_timeline.txt 2>&1 || true
cat gpurun_out/r6t_timeline.txt
echo CALL16DONE
