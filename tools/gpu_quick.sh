# Quick GPU check: SDWA probe, extractor parity suite, short bench (no CPU baseline).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -x tools/sdwa_probe ]; then timeout -k 5 60 ./tools/sdwa_probe > gpurun_out/sdwa.log 2>&1; fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bq.log 2>&1
echo DONE
