set -o pipefail
# round-5 final bench lines (one build), each under its own limit
OUT=gpurun_out/${1:-r05_final6}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
echo "default done"
for c in C D F G H N; do
timeout -k 10 400 python bench.py --config $c --no-cpu-baseline --no-side-mode > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 1
echo "$c done"
done
