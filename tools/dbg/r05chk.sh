set -o pipefail
OUT=gpurun_out/r05chk; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 python bench.py --config H --no-cpu-baseline --no-side-mode > $OUT/bench_H.json 2> $OUT/bench_H.err || exit 1
echo "H done"
timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline --no-side-mode > $OUT/bench_B5.json 2> $OUT/bench_B5.err || exit 1
echo "B done"
PBRT_PATHS_OVERLAP=0 timeout -k 10 200 python bench.py --steps 5 --no-cpu-baseline --no-side-mode > $OUT/bench_B5_noov.json 2> $OUT/bench_B5_noov.err || exit 1
echo "B noov done"
