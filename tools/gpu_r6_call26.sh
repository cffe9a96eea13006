# Round-6 call 26: the MFMA blur at 48 VGPRs (tap tables per column tile, the
# staged patch pre-biased to signed bytes, signed moments, tiles serialised):
# the -m gpu suite, then default vs 4 waves per block (liborbgpu_w4) vs the VALU
# blur (liborbgpu_base); bench + VALU PMC.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6ae}
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/${tag}_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; grep -E "FAILED|Error" gpurun_out/${tag}_tests.log | head -20; exit $rc; }
NO_PMC=1 ROUNDS=2 bash tools/gpu_r6_libab.sh ${tag} liborbgpu liborbgpu_w4 liborbgpu_base
for lib in liborbgpu liborbgpu_base; do
  ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY --output-format csv -d gpurun_out/${tag}_pmcv_${lib} -o q -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${tag}_pmcv_${lib}.log 2>&1 || { echo "pmc $lib failed"; exit 3; }
  python3 tools/pmc_summary.py gpurun_out/${tag}_pmcv_${lib}/q_counter_collection.csv > gpurun_out/${tag}_pmcv_${lib}.txt 2>&1 || true
done
echo CALL26DONE
