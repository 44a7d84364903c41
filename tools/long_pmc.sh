# SQ counters of the LONG string pass (phased vs row-order builds) on the 16..48-byte band (diagnostic)
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for lib in build_variants/libl0.so deequ_amd/libdqscan.so; do
  n=$(basename $lib .so)
  DQ_LIB_PATH=$GRAFT_REPO_ROOT/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d gpurun_out/r6l_pmc_$n -o p --output-format csv -- python3 tools/str_len_bench.py --path long --bands 16:48 --steps 1 > gpurun_out/r6l_pmc_$n.out 2>&1
done
