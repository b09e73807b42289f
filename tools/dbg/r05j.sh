set -o pipefail
OUT=gpurun_out/r05j; mkdir -p $OUT; export TMPDIR=/tmp
V=go-pbrt_amd/lib/exp/libpbrt_gpu_succdiag.so
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "filter or fullsize or lowdims or edges" > $OUT/pytest_film.log 2>&1 || { echo "film tests failed"; tail -30 $OUT/pytest_film.log; exit 1; }
echo "film tests done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o ks -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-side-mode > $OUT/ks.log 2>&1 && echo "ks done" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ksC -o ks -- python3 bench.py --config C --steps 1 --warmup 0 --no-cpu-baseline --no-side-mode > $OUT/ksC.log 2>&1 && echo "ksC done" &&
PBRT_GPU_LIB=$V timeout -k 10 300 python tools/heavy_tile.py --tiles 5389,4648 --waves 4 > $OUT/heavy_succdiag.txt 2>&1 && echo "heavy succdiag done" &&
PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_filmv3.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks3 -o ks -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-side-mode > $OUT/ks3.log 2>&1 && echo "ks3 done" &&
PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_filmv3.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "filter or fullsize or lowdims" > $OUT/pytest_film3.log 2>&1 && echo "film3 tests done"
