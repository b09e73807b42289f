set -o pipefail
OUT=gpurun_out/r05ov; mkdir -p $OUT; export TMPDIR=/tmp
V=go-pbrt_amd/lib/exp/libpbrt_gpu_ovp.so
timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline --no-side-mode > $OUT/bench_B_main.json 2> $OUT/bench_B_main.err || exit 1
echo "main done"
for t in 0 20 100 500; do
PBRT_GPU_LIB=$V PBRT_PATHS_OVERLAP=$t timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline --no-side-mode > $OUT/bench_B_ov$t.json 2> $OUT/bench_B_ov$t.err || exit 1
echo "ov$t done"
done
PBRT_GPU_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "paths_overlap" > $OUT/pytest_ov.log 2>&1 || { echo "tests failed"; tail -20 $OUT/pytest_ov.log; exit 1; }
echo "tests done"
