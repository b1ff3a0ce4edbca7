set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; o=gpurun_out/r03c5; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5.py tests/test_gpu_conn_keys.py -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1; tail -2 $o/pytest.log; grep -q " passed" $o/pytest.log && ! grep -q "failed" $o/pytest.log || exit 1
for r in 1 2; do timeout -k 10 240 python bench.py --mode e2e --keys 4096 --rotate --packets 2097152 --steps 6 --warmup 2 --no-cpu > $o/c5_$r.json 2>$o/err.txt || { tail -5 $o/err.txt; exit 1; }; python -c "import json;d=json.load(open('$o/c5_$r.json'));print(d['value'],d['config']['rotate_ms_per_step'],d['config']['pipeline_ms_per_step'])"; done
timeout -k 10 240 python bench.py > $o/c2.json 2>$o/err.txt && python -c "import json;d=json.load(open('$o/c2.json'));print(d['value'],d['roofline'])"
