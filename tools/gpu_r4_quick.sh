# Round-4 quick check: the -m gpu tests of the files given (default: PnP,
# Initializer, adapter, launcher/host-fed), the box's CPU share as
# bench.cpu_info() sees it, then one default bench line without CPU legs.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
files=${@:-tests/test_pnp.py tests/test_init.py tests/test_adapter.py tests/test_bench_launch.py}
python3 -c "import bench, json; print(json.dumps(bench.cpu_info()))" > gpurun_out/${tag}_cpuinfo.json 2>&1
cat /proc/self/cgroup >> gpurun_out/${tag}_cpuinfo.json 2>&1 || true
timeout -k 10 600 python -u -m pytest $files -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1
echo QUICKDONE
