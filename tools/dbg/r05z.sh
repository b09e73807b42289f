set -o pipefail
OUT=gpurun_out/r05z; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline --no-side-mode > $OUT/bench_B_base.json 2> $OUT/bench_B_base.err || exit 1
echo "B base done"
PBRT_PATHS_OVERLAP=1 timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline --no-side-mode > $OUT/bench_B_ov.json 2> $OUT/bench_B_ov.err || exit 1
echo "B ov done"
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "paths_overlap" > $OUT/pytest_ov.log 2>&1 || { echo "tests failed"; tail -20 $OUT/pytest_ov.log; exit 1; }
echo "tests done"
