#!/bin/bash
# Builds tools/prim_bench_<name>.bin for dq_prim.hip sort variants (A/B on the GPU: tools/prim_bench_*.bin).
set -e
cd "$(dirname "$0")/.."
H=/opt/rocm/bin/hipcc
$H --offload-arch=gfx950 -O3 -std=c++17 -c tools/prim_bench.hip -o /tmp/pb.o
build() {  # name flags...
  local name=$1; shift
  $H --offload-arch=gfx950 -O3 -std=c++17 "$@" -c deequ_amd/csrc/dq_prim.hip -o /tmp/prim_$name.o
  $H --offload-arch=gfx950 /tmp/pb.o /tmp/prim_$name.o -o tools/prim_bench_$name.bin
}
build t512i16    -DDQ_SORT_THREADS=512 -DDQ_SORT_ITEMS=16 -DDQ_SORT_MAXWG=1024 &
build t512i16w512 -DDQ_SORT_THREADS=512 -DDQ_SORT_ITEMS=16 -DDQ_SORT_MAXWG=512 &
build t512i20    -DDQ_SORT_THREADS=512 -DDQ_SORT_ITEMS=20 -DDQ_SORT_MAXWG=1024 &
build t1024i8    -DDQ_SORT_THREADS=1024 -DDQ_SORT_ITEMS=8 -DDQ_SORT_MAXWG=1024 &
build t256i24    -DDQ_SORT_THREADS=256 -DDQ_SORT_ITEMS=24 -DDQ_SORT_MAXWG=1024 &
wait
