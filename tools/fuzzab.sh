#!/bin/bash
# fuzz A/B over library builds: 44 seeds each, failures counted (no -x).  usage: LIBS="ab/a.so ab/b.so" bash tools/fuzzab.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fuzzab
export QPP_FUZZ_EXTRA=${QPP_FUZZ_EXTRA:-40}
for lib in $LIBS; do
  n=$(basename $lib .so)
  QPP_LIB=$PWD/$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q --timeout 120 --timeout-method thread -k "random_operation" > gpurun_out/fuzzab/$n.log 2>&1
  rc=$?
  echo "$n rc $rc: $(tail -1 gpurun_out/fuzzab/$n.log)"
  [ $rc -le 1 ] || exit 1
done
