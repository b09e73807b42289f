set -o pipefail
OUT=gpurun_out/r05i; mkdir -p $OUT; export TMPDIR=/tmp
V=go-pbrt_amd/lib/exp/libpbrt_gpu_succ.so
PBRT_GPU_LIB=$V timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "waves or heavy or split or fullsize or cold or stride or materials or cornell or lowdims" > $OUT/pytest_succ.log 2>&1 || { echo "succ tests failed"; tail -30 $OUT/pytest_succ.log; exit 1; }
echo "succ tests done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o ks -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-side-mode > $OUT/ks.log 2>&1 && echo "ks done" &&
timeout -k 10 300 python tools/heavy_tile.py --tiles 5389,4648 --waves 2,4 > $OUT/heavy_base.txt 2>&1 && echo "heavy base done" &&
PBRT_GPU_LIB=$V timeout -k 10 300 python tools/heavy_tile.py --tiles 5389,4648 --waves 2,4 > $OUT/heavy_succ.txt 2>&1 && echo "heavy succ done" &&
PBRT_GPU_LIB=$V timeout -k 10 300 python bench.py --no-cpu-baseline --no-side-mode > $OUT/bench_B_succ.json 2> $OUT/bench_B_succ.err && echo "bench succ done" &&
timeout -k 10 300 python tools/shard_sim.py --ns 8 --ranks 0,1,2,3,4,5,6,7 > $OUT/shard8_base.txt 2>&1 && echo "shard base done" &&
PBRT_GPU_LIB=$V timeout -k 10 300 python tools/shard_sim.py --ns 8 --ranks 0,1,2,3,4,5,6,7 > $OUT/shard8_succ.txt 2>&1 && echo "shard succ done"
