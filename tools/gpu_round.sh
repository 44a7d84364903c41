#!/bin/bash
# gpu_round.sh TAG STEP [STEP ...] -- one gpurun call of GPU steps (replaces round 4's one-off r4_gpuN.sh scripts).
# Every step runs under its own time limit and writes gpurun_out/TAG_<step>.*; the call stops at the first
# failing step (no GPU step after a fault, abort or timeout).  Steps:
#   suite            the whole GPU test suite (pytest -m gpu)
#   test=PATHS       pytest over PATHS (comma-separated, e.g. tests/test_plan_split.py,tests/test_pair_lane.py)
#   smoke            __graft_entry__.smoke()
#   bench[=ARGS]     python bench.py ARGS (ARGS with ',' for spaces) -> TAG_bench.json
#   prof             tools/profile_round.sh TAG (kernel trace + FETCH + SQ passes of the default bench)
#   pmc5             tools/pmc_c5.sh TAG (SQ counter passes of the C5 headline kernels)
#   clock            tools/clock_probe.sh TAG (held clock under the headline kernels)
#   parity[=CFGS]    tests/fullscale_parity.py at 1e9 rows (CFGS e.g. c3,c5) -> TAG_parity.json
#   py=SCRIPT[,ARGS] python SCRIPT ARGS
#   sh=SCRIPT[,ARGS] bash SCRIPT ARGS (e.g. sh=tools/ab_c5.sh,build_variants/libgold.so,deequ_amd/libdqscan.so)
# Usage: /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/gpu_round.sh r5a test=tests/test_plan_split.py bench
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/${TAG}_summary.txt
: > "$S"
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
for step in "$@"; do
  name=${step%%=*}; arg=""; [ "$step" != "$name" ] && arg=${step#*=}
  echo "== $step" | tee -a "$S"
  case $name in
    suite) timeout -k 10 900 $PYT tests -m gpu > gpurun_out/${TAG}_suite.log 2>&1
           rc=$?; tail -3 gpurun_out/${TAG}_suite.log | tee -a "$S" ;;
    test)  timeout -k 10 600 $PYT ${arg//,/ } > gpurun_out/${TAG}_test.log 2>&1
           rc=$?; tail -3 gpurun_out/${TAG}_test.log | tee -a "$S" ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
             > gpurun_out/${TAG}_smoke.txt 2>&1
           rc=$?; tail -2 gpurun_out/${TAG}_smoke.txt | tee -a "$S" ;;
    bench) timeout -k 10 600 python -u bench.py ${arg//,/ } > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
           rc=$?; tail -c 600 gpurun_out/${TAG}_bench.json | tee -a "$S"; echo >> "$S" ;;
    prof)  timeout -k 10 1100 bash tools/profile_round.sh "$TAG" > gpurun_out/${TAG}_prof.txt 2>&1
           rc=$?; tail -5 gpurun_out/${TAG}_prof.txt | tee -a "$S" ;;
    pmc5)  timeout -k 10 600 bash tools/pmc_c5.sh "${TAG}_pmc5" > gpurun_out/${TAG}_pmc5.out 2>&1
           rc=$?; tail -30 gpurun_out/${TAG}_pmc5.out | tee -a "$S" ;;
    clock) timeout -k 10 400 bash tools/clock_probe.sh "${TAG}_clock" > gpurun_out/${TAG}_clock.txt 2>&1
           rc=$?; tail -10 gpurun_out/${TAG}_clock.txt | tee -a "$S" ;;
    parity) timeout -k 10 1000 python -u tests/fullscale_parity.py ${arg:+--cfg ${arg//,/ }} \
              --out gpurun_out/${TAG}_parity.json > gpurun_out/${TAG}_parity.txt 2>&1
           rc=$?; tail -5 gpurun_out/${TAG}_parity.txt | tee -a "$S" ;;
    py)    timeout -k 10 600 python -u ${arg//,/ } > gpurun_out/${TAG}_py.txt 2>&1
           rc=$?; tail -20 gpurun_out/${TAG}_py.txt | tee -a "$S" ;;
    sh)    TAG=${TAG}_sh timeout -k 10 900 bash ${arg//,/ } > gpurun_out/${TAG}_sh.txt 2>&1
           rc=$?; tail -20 gpurun_out/${TAG}_sh.txt | tee -a "$S" ;;
    *)     echo "unknown step $step" | tee -a "$S"; exit 2 ;;
  esac
  [ $rc -eq 0 ] || { echo "step $step failed rc=$rc" | tee -a "$S"; exit $rc; }
done
echo "all steps ok" | tee -a "$S"
