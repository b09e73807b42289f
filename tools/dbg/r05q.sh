set -o pipefail
OUT=gpurun_out/r05q; mkdir -p $OUT; export TMPDIR=/tmp
export PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_widec.so
timeout -k 10 400 python bench.py --config D --steps 2 --no-cpu-baseline --no-side-mode > $OUT/bench_D_widec.json 2> $OUT/bench_D_widec.err || exit 1
echo "D widec done"
timeout -k 10 500 python -u -m pytest tests/test_gpu_mesh.py -x -q --timeout 300 --timeout-method thread -k "not config_E" > $OUT/mesh_tests.log 2>&1 || { echo "mesh tests failed"; tail -30 $OUT/mesh_tests.log; exit 1; }
echo "mesh tests done"
