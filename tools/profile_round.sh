#!/bin/bash
# profile_round.sh <tag> -- rocprofv3 evidence for bench.py on the GPU box (run via gpurun):
#   1. kernel trace + stats of the default bench workload (C5, 1e9 rows, 8 chunks of 125 M rows)
#   2. FETCH_SIZE pass (its own run, no tracing domains besides the counters), 4 chunks
#   3. SQ instruction-count pass (VALU / VMEM / LDS instructions per kernel), 4 chunks
# then tools/summarize_prof.py writes profiles/<tag>_*.  Stops at the first failing step.
set -u
TAG=${1:-r1}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out profiles
export TMPDIR=/tmp
B="bench.py --cpu-sample 0 --configs= --ingest-rows 0"
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt --output-format csv -- \
  python3 $B --steps 3 --warmup 1 > gpurun_out/prof_kt_bench.json 2> gpurun_out/prof_kt.err || { echo "kt failed $?"; tail -20 gpurun_out/prof_kt.err; exit 2; }
echo "kt ok"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_pmc -o pmc --output-format csv -- \
  python3 $B --rows 250000000 --steps 1 --warmup 0 > gpurun_out/prof_pmc_bench.json 2> gpurun_out/prof_pmc.err || { echo "pmc failed $?"; tail -20 gpurun_out/prof_pmc.err; exit 3; }
echo "pmc ok"
python3 tools/summarize_prof.py "$TAG" gpurun_out/prof_kt gpurun_out/prof_pmc || exit 4
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES -d gpurun_out/prof_sq -o sq --output-format csv -- \
  python3 $B --rows 250000000 --steps 1 --warmup 0 > gpurun_out/prof_sq_bench.json 2> gpurun_out/prof_sq.err || { echo "sq failed $?"; tail -20 gpurun_out/prof_sq.err; exit 5; }
echo "sq ok"
python3 tools/summarize_prof.py "$TAG" gpurun_out/prof_kt gpurun_out/prof_pmc gpurun_out/prof_sq
