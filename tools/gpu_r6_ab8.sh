# Round-6 call 8: the whole -m gpu suite on the default build (FAST window staged
# column-shifted so the detection region starts 4-aligned: 8 compass groups per
# 30-32 px row; staging loads as global_load with a scalar base), then default
# vs the HEAD build before it (liborbgpu_base), bench + a VALU PMC pass each.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6i}
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/${tag}_tests.log 2>&1 || { rc=$?; echo "tests rc=$rc"; [ $rc -eq 1 ] || exit $rc; }
NO_PMC=1 ROUNDS=3 bash tools/gpu_r6_libab.sh ${tag} liborbgpu liborbgpu_base
for lib in liborbgpu liborbgpu_base; do
  ORBGPU_LIBRARY=orb-slam2-annotation_amd/$lib.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/${tag}_pmcv_${lib} -o q -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${tag}_pmcv_${lib}.log 2>&1 || { echo "pmc $lib failed"; exit 3; }
  python3 tools/pmc_summary.py gpurun_out/${tag}_pmcv_${lib}/q_counter_collection.csv > gpurun_out/${tag}_pmcv_${lib}.txt 2>&1 || true
done
echo AB8DONE
