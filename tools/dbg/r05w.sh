set -o pipefail
OUT=gpurun_out/r05w; mkdir -p $OUT; export TMPDIR=/tmp
export PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_rrn.so
timeout -k 10 200 python bench.py --config G --steps 3 --no-cpu-baseline --no-side-mode > $OUT/bench_G_rrn.json 2> $OUT/bench_G_rrn.err || exit 1
echo "G rrn done"
timeout -k 10 600 python -u -m pytest tests/test_materials.py tests/test_fixtures_materials.py tests/test_gpu_lowdims.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_kx.log 2>&1 || { echo "kx tests failed"; tail -20 $OUT/pytest_kx.log; exit 1; }
echo "kx tests done"
unset PBRT_GPU_LIB
timeout -k 10 200 python bench.py --config G --steps 3 --no-cpu-baseline --no-side-mode > $OUT/bench_G_main.json 2> $OUT/bench_G_main.err || exit 1
echo "G main done"
