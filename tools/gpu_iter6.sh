set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in p16 p64 p128; do
  ORBGPU_LIBRARY=$PWD/exp/$v/liborbgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "pyramid or blurred or keypoints" --timeout 120 --timeout-method thread > gpurun_out/par_$v.log 2>&1 || { echo "$v PARITY FAIL"; tail -3 gpurun_out/par_$v.log; }
done
bash tools/variants_kstats.sh
for v in p16 p128; do
  export ORBGPU_LIBRARY=$PWD/exp/$v/liborbgpu.so
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/vf_$v -o f -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2>&1
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/vw_$v -o w -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2>&1
  python3 tools/make_traffic.py gpurun_out/vf_$v/f_counter_collection.csv gpurun_out/vw_$v/w_counter_collection.csv --out gpurun_out/tr_$v.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', 'read', round(d['read_bytes_corrected']/1e6), 'MB write', round(d['write_bytes']/1e6), 'MB')"
done
