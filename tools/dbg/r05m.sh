set -o pipefail
OUT=gpurun_out/r05m; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "mesh or lowdims" > $OUT/pytest_mesh.log 2>&1 || { echo "mesh tests failed"; tail -30 $OUT/pytest_mesh.log; exit 1; }
echo "mesh tests done"
timeout -k 10 400 python bench.py --config D --steps 2 --no-cpu-baseline --no-side-mode > $OUT/bench_D.json 2> $OUT/bench_D.err && echo "D done" &&
PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_nobatch.so timeout -k 10 400 python bench.py --config D --steps 2 --no-cpu-baseline --no-side-mode > $OUT/bench_D_nobatch.json 2> $OUT/bench_D_nobatch.err && echo "D nobatch done"
