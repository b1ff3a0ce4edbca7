#!/bin/bash
# One parameterized runner for GPU-box work (replaces the per-step tools/r03/*, tools/r04/* scripts).
#
# usage (on the GPU box, through gpurun):  bash tools/gpu.sh <tag> <step> [<step> ...]
#   each <step> is ONE shell word "name[:arg arg ...]" (quote it); steps run in order, the first failure ends the call.
#   outputs go to gpurun_out/<tag>/.
#
# steps
#   tests[:pytest args]       pytest -m gpu (default: the whole GPU suite) -> pytest.log
#   smoke                     __graft_entry__.smoke() -> smoke.log
#   bench[:name bench args]   python bench.py <args> -> <name>.json (name defaults to "bench")
#   ab[:sub CFGS|ARGS]        tools/ab.sh (same-box alternating A/B); CFGS and bench args separated by '|'
#                             e.g. "ab:aad ab/x.so:x s2n-quic_amd/libqpp.so:new|--aad 32"
#   pmcab[:sub LIBS|ARGS]     tools/pmc_ab.sh: FETCH_SIZE / WRITE_SIZE per library build (same box), LIBS and bench args
#                             separated by '|', e.g. "pmcab:nt s2n-quic_amd/libqpp.so ab/nt0.so"
#   prof[:bench args]         rocprofv3 kernel trace + PMC passes (tools/profile.sh) -> gpurun_out/<tag>_prof,
#                             then prof_summary.txt and traffic.json of the default workload in gpurun_out/<tag>/
#   rxtrace                   rocprofv3 kernel trace of the fused receive (exit status recorded)
#   matrix                    tools/bench_matrix.sh: every BASELINE config and mode -> gpurun_out/<tag>_matrix/
#   lat                       the latency faces: per-packet seal/open (AES, ChaCha), 64-packet txq flush (AES, ChaCha)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd $(dirname $0)/.. && pwd)}"
export TMPDIR=/tmp
tag=$1; shift
o=gpurun_out/$tag; mkdir -p $o
run_json() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $o/$name.json 2> $o/$name.err || { echo "FAIL $name"; tail -8 $o/$name.err; return 1; }
  echo "$name: $(head -c 400 $o/$name.json)"
}
for step in "$@"; do
  name=${step%%:*}; args=""; [ "$name" != "$step" ] && args=${step#*:}
  case $name in
    tests)
      timeout -k 10 600 python -u -m pytest ${args:-tests -m gpu} -q -x --timeout 120 --timeout-method thread > $o/pytest.log 2>&1
      rc=$?; tail -4 $o/pytest.log; [ $rc -eq 0 ] || exit 1 ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
      tail -3 $o/smoke.log ;;
    bench)
      set -- $args; bname=${1:-bench}; [ $# -gt 0 ] && shift
      run_json $bname 300 python bench.py "$@" || exit 1 ;;
    ab)
      sub=${args%% *}; rest=${args#* }; cfgs=${rest%%|*}; bargs=""; [[ "$rest" == *"|"* ]] && bargs=${rest#*|}
      CFGS="$cfgs" BENCH_ARGS="$bargs" bash tools/ab.sh ${tag}_$sub || exit 1 ;;
    pmcab)
      sub=${args%% *}; rest=${args#* }; libs=${rest%%|*}; bargs=""; [[ "$rest" == *"|"* ]] && bargs=${rest#*|}
      LIBS="$libs" BENCH_ARGS="$bargs" bash tools/pmc_ab.sh ${tag}_$sub || exit 1 ;;
    prof)
      bash tools/profile.sh ${tag}_prof $args || exit 1
      python tools/summarize_prof.py gpurun_out/${tag}_prof > $o/prof_summary.txt && head -14 $o/prof_summary.txt || exit 1
      if [ -z "$args" ]; then python tools/traffic.py gpurun_out/${tag}_prof aes128gcm/1200/1 1048576 $o/traffic.json || exit 1; fi ;;
    rxtrace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/rxtrace -o trace -- python3 bench.py --mode rx --keys 64 --steps 4 --warmup 1 --no-cpu > $o/rxtrace.log 2>&1
      rc=$?; echo "rx trace exit $rc" | tee $o/rxtrace.rc; [ $rc -eq 0 ] || exit 1 ;;
    matrix)
      bash tools/bench_matrix.sh ${tag}_matrix || exit 1 ;;
    lat)
      run_json packet_aes 120 python bench.py --mode packet --no-cpu && \
      run_json packet_chacha 120 python bench.py --mode packet --suite chacha20poly1305 --no-cpu && \
      run_json txq1_aes 120 python bench.py --mode txq --inflight 1 --no-cpu && \
      run_json txq1_chacha 120 python bench.py --mode txq --suite chacha20poly1305 --inflight 1 --no-cpu || exit 1 ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
