# Round-6 call 22: describe's blur on the matrix cores (row pass i8 MFMA, column
# pass f16 MFMA; ORBGPU_DESC_MFMA=1, the default) -- the whole -m gpu suite, then
# default vs the VALU blur (liborbgpu_base: -DORBGPU_DESC_MFMA=0), bench + VALU PMC.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6aa}
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/${tag}_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/${tag}_tests.log; exit $rc; }
NO_PMC=1 ROUNDS=3 bash tools/gpu_r6_libab.sh ${tag} liborbgpu liborbgpu_base
for lib in liborbgpu liborbgpu_base; do
  ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/${tag}_pmcv_${lib} -o q -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${tag}_pmcv_${lib}.log 2>&1 || { echo "pmc $lib failed"; exit 3; }
  python3 tools/pmc_summary.py gpurun_out/${tag}_pmcv_${lib}/q_counter_collection.csv > gpurun_out/${tag}_pmcv_${lib}.txt 2>&1 || true
done
echo CALL22DONE
