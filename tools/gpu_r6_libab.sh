# Round-6 library A/B: for each library named, the bench line (no extras / CPU
# legs, 40 timed steps after 20 warm-up steps) interleaved over $ROUNDS rounds,
# then one PMC pass per library (FETCH_SIZE, LDS bank conflicts, CU-busy cycles)
# over a short bench.   usage: ROUNDS=2 bash tools/gpu_r6_libab.sh <tag> lib1 lib2 ...
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --steps 40 --warmup 20 > gpurun_out/${tag}_${lib}_$r.log 2>&1 || { echo "$lib failed"; exit 3; }
  done
done
if [ -z "$NO_PMC" ]; then
  for lib in "$@"; do
    ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/${tag}_pmc_${lib} -o q -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${tag}_pmc_${lib}.log 2>&1 || { echo "pmc $lib failed"; exit 3; }
    python3 tools/pmc_summary.py gpurun_out/${tag}_pmc_${lib}/q_counter_collection.csv > gpurun_out/${tag}_pmc_${lib}.txt 2>&1 || true
  done
fi
echo LIBABDONE
