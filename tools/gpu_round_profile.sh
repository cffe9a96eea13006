# One GPU call: GPU parity suite, FETCH_SIZE / WRITE_SIZE PMC passes ->
# profiles/pmc_traffic.json, default bench (with CPU baseline), rocprofv3
# kernel stats.  Results under gpurun_out/ (copied to profiles/ by hand).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pf -o pf -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pf.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pw -o pw -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pw.log 2>&1
python3 tools/make_traffic.py gpurun_out/pf/pf_counter_collection.csv gpurun_out/pw/pw_counter_collection.csv --config mono640 --batch 512 --algorithmic 803777536 --out gpurun_out/pmc_traffic.json > gpurun_out/traffic.log 2>&1
timeout -k 10 300 python bench.py --traffic-json gpurun_out/pmc_traffic.json > gpurun_out/bench_full.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks -o ks -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ks.log 2>&1
echo ALLDONE
