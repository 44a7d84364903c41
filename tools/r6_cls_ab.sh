#!/bin/bash
# Round-6 A/B of the string pass by stripe-count class (DQ_STR_CLS) against the round-5 loop:
# GPU tests of the string hash with the class build, C5 headline alternating the two builds on one box, then SQ /
# TCP counter passes of both (VALU per launch, L1 -> L2 read requests).  Usage (GPU box):
#   bash tools/r6_cls_ab.sh TAG OLD.so NEW.so
set -u
TAG=$1; OLD=$2; NEW=$3
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
DQ_LIB_PATH=$NEW timeout -k 10 600 python -u -m pytest tests/test_utf8_hll.py tests/test_hll_redo.py tests/test_gpu_parity.py \
  tests/test_types_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG}_c5 STEPS=8 bash tools/ab_c5.sh $OLD $NEW $OLD $NEW || exit $?
export PASSES="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT;TCP_TCC_READ_REQ TCP_TOTAL_CACHE_ACCESSES TA_TA_BUSY GRBM_GUI_ACTIVE"
for lib in $OLD $NEW; do
  bash tools/pmc_c5.sh ${TAG}_pmc_$(basename $lib .so) $lib > /dev/null || exit $?
  echo "== $lib"; grep -E "utf8|column_scan<10" gpurun_out/${TAG}_pmc_$(basename $lib .so).txt | head -20
done
