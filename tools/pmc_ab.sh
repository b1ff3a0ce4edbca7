#!/bin/bash
# Same-box HBM traffic A/B: FETCH_SIZE and WRITE_SIZE passes (one counter group per rocprofv3 run) of a short bench
# for each library build, summarised per kernel by tools/pmc_sum.py.
# usage: LIBS="ab/a.so ab/b.so" [BENCH_ARGS=...] bash tools/pmc_ab.sh tag
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=${1:-pmcab}; mkdir -p gpurun_out/$tag
for lib in $LIBS; do
  n=$(basename $lib .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    QPP_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/$tag/$n/$c -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu $BENCH_ARGS > gpurun_out/$tag/$n.$c.log 2>&1 || { echo "pmc $n $c failed"; tail -5 gpurun_out/$tag/$n.$c.log; exit 1; }
  done
  python3 tools/pmc_sum.py gpurun_out/$tag/$n quad_kernel
done
