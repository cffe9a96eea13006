# Drop-in transfers by kernels vs the copy engine: the adapter and extractor
# parity tests, every drop-in latency (tools/dropin_profile.py) with the copy
# kernels (default) and with ORBGPU_HOST_ZEROCOPY=0 ORBGPU_SINGLE_ZEROCOPY=0,
# then the sub-batch bench legs.  usage: bash tools/gpu_r4_dropin2.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_adapter.py tests/test_gpu_parity.py > gpurun_out/${tag}_tests.log 2>&1
timeout -k 10 300 python3 -u tools/dropin_profile.py 100 > gpurun_out/${tag}_dropin_kernels.json 2> gpurun_out/${tag}_dropin_kernels.err
ORBGPU_HOST_ZEROCOPY=0 ORBGPU_SINGLE_ZEROCOPY=0 timeout -k 10 300 python3 -u tools/dropin_profile.py 100 > gpurun_out/${tag}_dropin_sdma.json 2> gpurun_out/${tag}_dropin_sdma.err
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras > gpurun_out/${tag}_base.log 2>&1
for pp in "2 fast_cells" "2 pyramid"; do
  set -- $pp
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-extras --parts $1 --part-stage $2 > gpurun_out/${tag}_parts$1_$2.log 2>&1 || echo "parts $pp rc $?"
done
echo D2DONE
