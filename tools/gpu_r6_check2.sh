# Round-6 checkpoint at HEAD: every -m gpu test, smoke(), the full default bench
# line, then the single-frame kernels of the default build vs liborbgpu_base
# (kernel traces of the python probe) and the C++ drop-in extraction latency.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6q}
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/${tag}_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/${tag}_tests.log; exit $rc; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/${tag}_smoke.log 2>&1
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/${tag}_bench.log 2>&1
tail -c 300 gpurun_out/${tag}_bench.log
ROUNDS=0 bash tools/gpu_r6_single3.sh ${tag}_new new:liborbgpu
ROUNDS=0 bash tools/gpu_r6_single3.sh ${tag}_base base:liborbgpu_base
ROUNDS=2 REPS=1000 timeout -k 10 600 python3 -u tools/extract_cpp_probe.py new > gpurun_out/${tag}_cpp.txt 2>&1 || { echo "cpp probe failed"; exit 3; }
cat gpurun_out/${tag}_cpp.txt
echo CHECK2DONE
