#!/bin/bash
# memory-path counters (TA / TCP / TCC), one rocprofv3 pass per counter group
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=${1:-mem}; shift
out=gpurun_out/$tag; mkdir -p $out
B="python3 bench.py --steps 2 --warmup 1 --no-cpu $*"
i=0
for pmc in "TA_BUSY_sum GRBM_GUI_ACTIVE" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TCC_HIT_sum TCC_MISS_sum" "TD_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc$i -o pmc -- $B > $out/pmc$i.log 2>&1 || { echo "pmc pass $i ($pmc) failed"; tail -5 $out/pmc$i.log; }
done
echo done
