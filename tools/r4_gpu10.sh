#!/bin/bash
# round-4 GPU call 10 (final evidence, part 1): rocprofv3 kernel trace + stats, FETCH_SIZE and SQ passes of the default
# bench workload (tools/profile_round.sh r4z), then the held-clock probe of the headline kernels (tools/clock_probe.sh)
# and of C3 / C4.  Everything lands in gpurun_out/ (profiles/ on the box does not come back).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out/r4z_profiles
export TMPDIR=/tmp
bash tools/profile_round.sh r4z > gpurun_out/r4z_profile_round.log 2>&1
rc=$?; cp profiles/r4z_* gpurun_out/r4z_profiles/ 2>/dev/null; tail -3 gpurun_out/r4z_profile_round.log; [ $rc -eq 0 ] || exit $rc
bash tools/clock_probe.sh r4z_clk > gpurun_out/r4z_clk.log 2>&1 || { tail -5 gpurun_out/r4z_clk.log; exit 4; }
python3 tools/clock_summary.py gpurun_out/r4z_clk gpurun_out/r4z_profiles/r4z_clock.json > /dev/null || exit 5
CFG=c3,c4 ROWS=250000000 bash tools/clock_probe.sh r4z_clkcfg > gpurun_out/r4z_clkcfg.log 2>&1 || { tail -5 gpurun_out/r4z_clkcfg.log; exit 6; }
python3 tools/clock_summary.py gpurun_out/r4z_clkcfg gpurun_out/r4z_profiles/r4z_cfg_clock.json > /dev/null || exit 7
ls gpurun_out/r4z_profiles
