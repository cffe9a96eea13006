# A/B of the pyramid kernels: parity suite and per-kernel times per mode
# (ORBGPU_PYR_MODE = stream (default) | frame | band).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in ${MODES:-stream frame band}; do
  ORBGPU_PYR_MODE=$m timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/par_$m.log 2>&1 || { echo "$m PARITY FAIL"; tail -5 gpurun_out/par_$m.log; exit 1; }
  ORBGPU_PYR_MODE=$m timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_$m -o ab -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$m.log 2>&1
  python3 - "$m" gpurun_out/ab_$m/ab_kernel_stats.csv <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[2])) if "pyramid" in r["Name"]]
print(sys.argv[1], "parity ok", " ".join(f"{r['Name'].split('::')[-1].split('(')[0][:22]}={float(r['AverageNs'])/1e3:.1f}us" for r in rows))
PY
done
