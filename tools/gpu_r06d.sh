# quad vs wave kernel crossover in packets per key (round 6 item 4), and the receive path's kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/r06d; mkdir -p $o
export TMPDIR=/tmp
b() { n=$1; shift; timeout -k 10 200 "$@" > $o/$n.json 2> $o/$n.err || { echo "FAIL $n"; tail -5 $o/$n.err; return 1; }; python3 -c "import json,sys; d=json.load(open('$o/$n.json')); c=d.get('config',{}); print('$n', d['value'], c.get('seal_ms'), c.get('open_ms'))"; }
for kp in "4096 262144" "4096 524288" "4096 1048576" "4096 2097152" "1024 1048576" "16384 2097152"; do
  set -- $kp
  QPP_AES_KERNEL=quad b q_k$1_n$2 python bench.py --no-cpu --steps 5 --warmup 2 --keys $1 --packets $2 || exit 1
  QPP_AES_KERNEL=wave b w_k$1_n$2 python bench.py --no-cpu --steps 5 --warmup 2 --keys $1 --packets $2 || exit 1
done
b k1_1mi python bench.py --no-cpu --steps 5 --warmup 2 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_rx1 -o trace -- python3 bench.py --no-cpu --steps 3 --warmup 1 --mode rx --keys 1 > $o/tr_rx1.log 2>&1 && \
echo done
