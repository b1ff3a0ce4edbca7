#!/bin/bash
# rocprofv3 passes over a short bench run (kernel trace + separate PMC passes, as MI355X_MICROARCH.md prescribes).
# usage: bash tools/profile.sh <tag> [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=${1:-prof}; shift
out=gpurun_out/$tag
mkdir -p $out
B="python3 bench.py --steps 4 --warmup 1 --no-cpu $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o trace -- $B > $out/trace.log 2>&1 || { echo "trace failed"; tail -20 $out/trace.log; exit 1; }
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc$i -o pmc -- $B > $out/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $out/pmc$i.log; exit 1; }
done
echo "profile done: $out"
