# Iteration check: extractor parity suite on the product build, then
# per-kernel timing of every exp/* variant (tools/pyr_variants.sh).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1
bash tools/variants_kstats.sh
