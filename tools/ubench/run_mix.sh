#!/bin/bash
# tools/ubench/mix on the GPU box: timings, then two rocprofv3 PMC passes (each its own run), then the per-kernel
# pipe fractions (tools/ubench/mix_pmc.py).  usage: bash tools/ubench/run_mix.sh <outdir> [mode]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd $(dirname $0)/../.. && pwd)}"
export TMPDIR=/tmp
o=${1:-gpurun_out/mix}; mode=${2:-all}; mkdir -p $o
timeout -k 10 180 ./tools/ubench/mix $mode > $o/mix.txt 2>&1 || { echo "mix failed"; tail $o/mix.txt; exit 1; }
cat $o/mix.txt
i=0
for pmc in "SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --output-format csv -d $o/pmc$i -o pmc -- ./tools/ubench/mix $mode > $o/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail $o/pmc$i.log; exit 1; }
done
python3 tools/ubench/mix_pmc.py $o | tee $o/mix_pmc.txt
