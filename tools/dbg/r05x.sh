set -o pipefail
OUT=gpurun_out/r05x; mkdir -p $OUT; export TMPDIR=/tmp
export PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_psplit.so
timeout -k 10 200 python bench.py --steps 2 --no-cpu-baseline --no-side-mode > $OUT/bench_B_psplit.json 2> $OUT/bench_B_psplit.err || exit 1
echo "B psplit done"
PBRT_CI_PROBE_HEAVY=16 timeout -k 10 200 python bench.py --steps 2 --no-cpu-baseline --no-side-mode > $OUT/bench_B_psplit16.json 2> $OUT/bench_B_psplit16.err || exit 1
echo "B psplit16 done"
PBRT_CI_PROBE_HEAVY=128 timeout -k 10 200 python bench.py --steps 2 --no-cpu-baseline --no-side-mode > $OUT/bench_B_psplit128.json 2> $OUT/bench_B_psplit128.err || exit 1
echo "B psplit128 done"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "split or cold_frame or config_B_whole_frame" > $OUT/pytest_split.log 2>&1 || { echo "tests failed"; tail -20 $OUT/pytest_split.log; exit 1; }
echo "tests done"
