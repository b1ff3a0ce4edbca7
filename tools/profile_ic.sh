#!/bin/bash
# icache / ifetch counters for the bench kernels (separate PMC passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=${1:-ic}; shift
out=gpurun_out/$tag; mkdir -p $out
B="python3 bench.py --steps 3 --warmup 1 --no-cpu $*"
i=0
for pmc in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH GRBM_GUI_ACTIVE" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_IFETCH_LEVEL SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc$i -o pmc -- $B > $out/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $out/pmc$i.log; exit 1; }
done
echo done
