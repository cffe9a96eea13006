# Build tuning/diagnostic variants of liborbgpu.so into
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
    # FILES (env) = the sources the flags affect; the rest are reused from build/
    files=${FILES:-"pyramid.hip orbgpu.cpp"}
    objs=$(ls build/*.o)
    for f in $files; do
        case $f in *.hip) $H $flags -c csrc/$f -o $d/$f.o & ;; *) $H $flags -x hip -c csrc/$f -o $d/$f.o & ;; esac
        objs=$(echo "$objs" | grep -v "/$f.o")
    done
    wait
    $H -shared -o $d/liborbgpu.so $d/*.o $objs
    echo "built $d ($flags)"
done
