# One GPU call: GPU parity suite, default bench (with CPU baseline),
# rocprofv3 kernel stats, and the FETCH_SIZE / WRITE_SIZE PMC passes.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_all.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_full.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks -o ks -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ks.log 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pf -o pf -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pf.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pw -o pw -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pw.log 2>&1
echo ALLDONE
