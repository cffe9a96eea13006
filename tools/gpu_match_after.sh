# Where the matcher stream starts within the step: A/B of --match-after; plus smoke.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke.log 2>&1
for m in fast_cells octree pyramid fast_cells octree; do
  timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline --match-after $m > gpurun_out/ma_$m.log 2>&1
  grep -o '"value": [0-9.]*' gpurun_out/ma_$m.log | sed "s/^/$m /" >> gpurun_out/ma_summary.txt
done
echo MADONE
