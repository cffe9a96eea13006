set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a_gpu_all.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2a_bench.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2a_ks -o ks -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r2a_ks.log 2>&1
echo ALLDONE
