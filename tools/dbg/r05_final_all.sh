set -o pipefail
OUT=gpurun_out/${1:-r05_final17}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest.log; exit 1; }
echo "tests done"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
echo "smoke done"
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
echo "default done"
for c in C D F G H N; do
timeout -k 10 400 python bench.py --config $c --no-cpu-baseline --no-side-mode > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 1
echo "$c done"
done
