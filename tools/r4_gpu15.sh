#!/bin/bash
# round-4 GPU call 15: predicate-pass workgroups per chunk on C3 (in-tree 2048; 1024 = one round of resident
# workgroups; 4096; 8192) -- the compiled pass issues VALU at ~76 % of the held clock's rate while its waves look
# ~93 % busy when resident: is the rest the two-round tail?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=c3 SKIP_TESTS=1 TAG=r4o3 bash tools/ab_c3.sh deequ_amd/libdqscan.so build_variants/libpwg1024.so build_variants/libpwg4096.so build_variants/libpwg8192.so deequ_amd/libdqscan.so build_variants/libpwg1024.so build_variants/libpwg4096.so build_variants/libpwg8192.so | tee gpurun_out/r4o_summary.txt
