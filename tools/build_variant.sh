#!/bin/bash
# build_variant.sh NAME [extra hipcc flags...] -- diagnostic A/B build: $SRC (default dq_kernels) .hip with
# the extra flags, linked with the other in-tree objects (deequ_amd/build/*.o) into
# build_variants/libNAME.so (select it with DQ_LIB_PATH).
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p build_variants/$NAME
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result "$@" \
  -c deequ_amd/csrc/${SRC:-dq_kernels}.hip -o build_variants/$NAME/${SRC:-dq_kernels}.o
OBJS=$(ls deequ_amd/build/*.o | grep -v ${SRC:-dq_kernels}.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build_variants/lib$NAME.so build_variants/$NAME/${SRC:-dq_kernels}.o $OBJS -lhiprtc
python3 -c "import ctypes; ctypes.CDLL(\"build_variants/lib$NAME.so\")" && echo build_variants/lib$NAME.so
