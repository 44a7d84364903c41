#!/bin/bash
# round-4 GPU call 12: 1e9-row parity of C2 / C3 / C4 / C5 on the final kernels (tests/fullscale_parity.py: integer
# results bit-exact vs the C oracle, fp64 within 1e-12 strict of a double-double reference).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u tests/fullscale_parity.py --cfg c3 c5 c4 c2 --rows 1000000000 \
  --out gpurun_out/r4z_fullscale_parity.json > gpurun_out/r4z_fullscale_parity.txt 2>&1
rc=$?; grep '^{' gpurun_out/r4z_fullscale_parity.txt | cut -c1-300; exit $rc
