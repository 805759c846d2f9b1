# Build an experimental variant of libsspp_hip.so: bash tools/build_variant.sh NAME "-DFLAG=..."
# -> sspp_amd/lib/variants/libsspp_NAME.so (git-ignored, travels with gpurun; load with
#    SSPP_LIB_PATH=sspp_amd/lib/variants/libsspp_NAME.so)
set -e
cd "$(dirname "$0")/.."
NAME=$1; FLAGS=$2
OUT=build/variants/$NAME; mkdir -p $OUT sspp_amd/lib/variants
HIPCC=/opt/rocm/bin/hipcc
# the product's objects (and its source stamp, sspp_build_id) must be current: the variant links them
make -s -j8 sspp_amd/lib/libsspp_hip.so
$HIPCC -std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -DSSPP_SINGLE_TU $FLAGS -c sspp_amd/csrc/sspp_kernels.hip -o $OUT/k.o
$HIPCC --offload-arch=gfx950 -shared -fPIC -o sspp_amd/lib/variants/libsspp_$NAME.so $OUT/k.o build/obj/ces.o build/obj/planner.o build/obj/sspp_capi.o build/obj/mjcf.o build/obj/spline_host.o build/obj/sspp_hostapi.o build/obj/stamp.o
