# Round-6 call 40: describe's wave totals by two row-broadcast DPP adds and one
# readlane (instead of four readlanes): extraction parity tests, then default vs
# HEAD (liborbgpu_prev), 3 rounds, + VALU PMC of both.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6as}
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_adapter.py tests/test_stereo.py > gpurun_out/${tag}_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; grep -E "FAILED|Error" gpurun_out/${tag}_tests.log | head -20; exit $rc; }
NO_PMC=1 ROUNDS=3 bash tools/gpu_r6_libab.sh ${tag} liborbgpu liborbgpu_prev
for lib in liborbgpu liborbgpu_prev; do
  ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/${tag}_pmcv_${lib} -o q -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${tag}_pmcv_${lib}.log 2>&1 || { echo "pmc $lib failed"; exit 3; }
  python3 tools/pmc_summary.py gpurun_out/${tag}_pmcv_${lib}/q_counter_collection.csv > gpurun_out/${tag}_pmcv_${lib}.txt 2>&1 || true
done
echo CALL40DONE
