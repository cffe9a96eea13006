# Round-3 check c: drop-in latencies under rocprofv3 with one output set per
# process (the adapter runs as a child of bench.py's DropIn).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r3c}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_dk -o dk_%pid% -- python3 tools/dropin_profile.py 10 > gpurun_out/${tag}_dk.log 2>&1
echo ALLDONE
