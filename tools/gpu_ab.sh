# A/B of the pyramid kernels: probe, parity (default kernel), per-kernel times
# for the default and the ORBGPU_PYR_MODE=band kernel.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 5 60 ./tools/sdwa_probe > gpurun_out/sdwa.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1
for m in frame band; do
  ORBGPU_PYR_MODE=$m timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_$m -o ab -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$m.log 2>&1
  python3 - "$m" gpurun_out/ab_$m/ab_kernel_stats.csv <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[2])) if "orbgpu" in r["Name"]]
print(sys.argv[1], " ".join(f"{r['Name'].split('::')[-1].split('(')[0][:22]}={float(r['AverageNs'])/1e3:.0f}" for r in rows))
PY
done
