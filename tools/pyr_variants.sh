# Build tuning variants of liborbgpu.so (pyramid probes / LDS budgets) into
# exp/<name>/ -- CPU side; run them on the GPU with tools/pyr_variants_run.sh.
# usage: tools/pyr_variants.sh name:FLAGS [name:FLAGS ...]
#   e.g. probe1:-DPYR_PROBE=1 lds64:-DORBGPU_PYR_LDS_KB=64
set -e
cd "$(dirname "$0")/../orb-slam2-annotation_amd"
make -s -j8 liborbgpu.so
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -I../include"
for spec in "$@"; do
    name=${spec%%:*}; flags=${spec#*:}; flags=${flags//,/ }
    d=../exp/$name; mkdir -p $d
    $H $flags -c csrc/pyramid.hip -o $d/pyramid.hip.o &
    $H $flags -x hip -c csrc/orbgpu.cpp -o $d/orbgpu.cpp.o &
    wait
    objs=$(ls build/*.o | grep -v -e '/pyramid.hip.o' -e '/orbgpu.cpp.o')
    $H -shared -o $d/liborbgpu.so $d/pyramid.hip.o $d/orbgpu.cpp.o $objs
    echo "built $d ($flags)"
done
