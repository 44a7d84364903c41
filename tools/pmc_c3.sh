set -u
# SQ pass over one config's kernels (CFG, default c3; 250 M rows, one step), per library; output gpurun_out/${TAG:-pmc}_<lib>
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
# usage: bash tools/pmc_c3.sh [lib.so ...]  (default: the in-tree library)
for lib in "${@:-deequ_amd/libdqscan.so}"; do
  n=$(basename $lib .so)
  DQ_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM -d gpurun_out/${TAG:-pmc}_$n -o p --output-format csv -- python3 bench.py --skip-headline --configs=${CFG:-c3} --config-rows 250000000 --config-steps 1 --cpu-sample 0 --ingest-rows 0 > gpurun_out/${TAG:-pmc}_$n.out 2>&1 || { echo "fail $n"; tail -5 gpurun_out/${TAG:-pmc}_$n.out; exit 2; }
  echo "ok $n"
done
