#!/bin/bash
# Builds tools/prim_bench_<name>.bin for dq_prim.hip sort variants (compile-time knobs DQ_SORT_THREADS / DQ_SORT_ITEMS
# / DQ_SORT_MAXWG; the pass form is chosen at run time: DQ_SORT_SEGMENTED=1 forces reduce-then-scan) for A/B runs of
# tools/prim_bench.hip on the GPU.  profiles/r6v_prim_sort_ab.txt records the variants measured in round 6.
set -e
cd "$(dirname "$0")/.."
H=/opt/rocm/bin/hipcc
$H --offload-arch=gfx950 -O3 -std=c++17 -c tools/prim_bench.hip -o /tmp/pb.o
build() {  # name flags...
  local name=$1; shift
  $H --offload-arch=gfx950 -O3 -std=c++17 "$@" -c deequ_amd/csrc/dq_prim.hip -o /tmp/prim_$name.o
  $H --offload-arch=gfx950 /tmp/pb.o /tmp/prim_$name.o -o tools/prim_bench_$name.bin
}
build t512i16 -DDQ_SORT_THREADS=512 -DDQ_SORT_ITEMS=16 &
build t256i16 -DDQ_SORT_THREADS=256 -DDQ_SORT_ITEMS=16 &
build t1024i8 -DDQ_SORT_THREADS=1024 -DDQ_SORT_ITEMS=8 &
wait
