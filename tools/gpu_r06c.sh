# many-key / small-packet / receive-path measurements (round 6 items 4-6)
set -o pipefail
cd $GRAFT_REPO_ROOT
o=gpurun_out/r06c; mkdir -p $o
export TMPDIR=/tmp
b() { n=$1; shift; timeout -k 10 200 "$@" > $o/$n.json 2> $o/$n.err || { echo "FAIL $n"; tail -5 $o/$n.err; return 1; }; python3 -c "import json,sys; d=json.load(open('$o/$n.json')); c=d['config']; print('$n', d['value'], c.get('seal_ms'), c.get('open_ms'), d.get('kernel_roofline',{}).get('lds') if d.get('kernel_roofline') else None)"; }
b k1_2mi python bench.py --no-cpu --steps 5 --warmup 2 --keys 1 --packets 2097152 && \
b k4096_auto python bench.py --no-cpu --steps 5 --warmup 2 --keys 4096 --packets 2097152 && \
QPP_AES_KERNEL=quad b k4096_quad python bench.py --no-cpu --steps 5 --warmup 2 --keys 4096 --packets 2097152 && \
QPP_AES_KERNEL=wave b k4096_wave python bench.py --no-cpu --steps 5 --warmup 2 --keys 4096 --packets 2097152 && \
b k64 python bench.py --no-cpu --steps 5 --warmup 2 --keys 64 && \
b pt300 python bench.py --no-cpu --steps 5 --warmup 2 --pt 300 --packets 4194304 && \
b rx1 python bench.py --no-cpu --steps 5 --warmup 2 --mode rx --keys 1 && \
b rx64 python bench.py --no-cpu --steps 5 --warmup 2 --mode rx --keys 64 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_k4096 -o trace -- python3 bench.py --no-cpu --steps 3 --warmup 1 --keys 4096 --packets 2097152 > $o/tr_k4096.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/tr_rx1 -o trace -- python3 bench.py --no-cpu --steps 3 --warmup 1 --mode rx --keys 1 > $o/tr_rx1.log 2>&1 && \
echo done
