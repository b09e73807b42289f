set -o pipefail
OUT=gpurun_out/r05r; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python bench.py --config D --steps 2 --no-cpu-baseline --no-side-mode > $OUT/bench_D_f32.json 2> $OUT/bench_D_f32.err || exit 1
echo "D f32 done"
PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_widef.so timeout -k 10 400 python bench.py --config D --steps 2 --no-cpu-baseline --no-side-mode > $OUT/bench_D_widef.json 2> $OUT/bench_D_widef.err || exit 1
echo "D widef done"
timeout -k 10 600 python -u -m pytest tests/test_gpu_mesh.py tests/test_gpu_lowdims.py -x -q --timeout 300 --timeout-method thread -k "not config_E" > $OUT/mesh_tests.log 2>&1 || { echo "mesh tests failed"; tail -30 $OUT/mesh_tests.log; exit 1; }
echo "mesh tests done"
