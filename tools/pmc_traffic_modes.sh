# GPU side: HBM traffic (FETCH_SIZE, WRITE_SIZE passes) of the pyramid kernel per mode.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
for m in ${MODES:-stream band}; do
    export ORBGPU_PYR_MODE=$m
    timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/tf_$m -o tf -- $B > gpurun_out/tf_$m.log 2>&1
    timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/tw_$m -o tw -- $B > gpurun_out/tw_$m.log 2>&1
    python3 - $m gpurun_out/tf_$m/tf_counter_collection.csv gpurun_out/tw_$m/tw_counter_collection.csv <<'PY'
import csv, sys
def get(p, c):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(p)) if "pyramid" in r["Kernel_Name"] and r["Counter_Name"] == c]
    return max(v) if v else float("nan")
f = get(sys.argv[2], "FETCH_SIZE"); w = get(sys.argv[3], "WRITE_SIZE")
print(sys.argv[1], f"FETCH_SIZE {f:.0f} KB (x2 = {2*f/1024:.1f} MB read)  WRITE_SIZE {w:.0f} KB ({w/1024:.1f} MB)")
PY
done
