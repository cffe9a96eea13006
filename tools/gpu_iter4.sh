set -e
cd $GRAFT_REPO_ROOT
ORBGPU_PYR_MODE=band bash tools/variants_kstats.sh
