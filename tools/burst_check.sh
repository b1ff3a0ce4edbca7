#!/bin/bash
# Burst-kernel change: the parity tests that run it (burst path, txq, per-packet, FIPS, fuzz), then the latency A/B.
# usage: A=<so> B=<so> bash tools/burst_check.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
tag=${1:-burst}; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fips.py tests/test_gpu_fuzz.py tests/test_gpu_lifetime.py -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit 1
bash tools/lat_ab.sh ${tag}_lat
