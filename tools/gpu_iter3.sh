set -e
cd $GRAFT_REPO_ROOT
bash tools/variants_kstats.sh
rm -rf exp/nowait
rm -rf exp/base
mkdir -p exp/band && cp orb-slam2-annotation_amd/liborbgpu.so exp/band/
for p in 0 1 32; do :; done
ORBGPU_PYR_MODE=band bash tools/variants_kstats.sh
