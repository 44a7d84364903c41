#!/bin/bash
# build_variant.sh NAME [extra hipcc flags...] -- diagnostic A/B build: $SRC (default dq_kernels; a .hip
# kernel source, or a .cpp host source with EXT=cpp) with the extra flags, linked with the other in-tree
# objects (deequ_amd/build/*.o) into build_variants/libNAME.so (select it with DQ_LIB_PATH).
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
SRC=${SRC:-dq_kernels}
mkdir -p build_variants/$NAME
if [ "${EXT:-hip}" = cpp ]; then
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -ffp-contract=off -Ideequ_amd/build \
    -Ideequ_amd/csrc "$@" -c deequ_amd/csrc/$SRC.cpp -o build_variants/$NAME/$SRC.o
else
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result "$@" \
    -c deequ_amd/csrc/$SRC.hip -o build_variants/$NAME/$SRC.o
fi
OBJS=$(ls deequ_amd/build/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build_variants/lib$NAME.so build_variants/$NAME/$SRC.o $OBJS -lhiprtc
python3 -c "import ctypes; ctypes.CDLL(\"build_variants/lib$NAME.so\")" && echo build_variants/lib$NAME.so
