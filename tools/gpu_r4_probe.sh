# D2H path probe under rocprofv3 (kernel + memory-copy trace): does a pinned D2H copy run on an SDMA engine or as a blit kernel?
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
timeout -k 10 120 python3 tools/d2h_probe.py > gpurun_out/${tag}_d2h.json 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/${tag}_d2h -o d -- python3 tools/d2h_probe.py > gpurun_out/${tag}_d2h_prof.log 2>&1
echo PROBEDONE
