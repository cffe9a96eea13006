# Round-6 call 9: the whole -m gpu suite on the default build (FAST compass rows
# mask only on the last pass, arc bias folded into the window base; describe raw
# staging stores at 16*idx, wave totals on fused DPP adds, disc-table loads with
# scalar bases), then default vs the HEAD build (liborbgpu_base), bench + VALU PMC each.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6j}
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/${tag}_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; [ $rc -eq 1 ] || exit $rc; }
NO_PMC=1 ROUNDS=3 bash tools/gpu_r6_libab.sh ${tag} liborbgpu liborbgpu_base
for lib in liborbgpu liborbgpu_base; do
  ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/${tag}_pmcv_${lib} -o q -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${tag}_pmcv_${lib}.log 2>&1 || { echo "pmc $lib failed"; exit 3; }
  python3 tools/pmc_summary.py gpurun_out/${tag}_pmcv_${lib}/q_counter_collection.csv > gpurun_out/${tag}_pmcv_${lib}.txt 2>&1 || true
done
echo AB9DONE
