set -o pipefail
OUT=gpurun_out/r05u; mkdir -p $OUT; export TMPDIR=/tmp
T=go-pbrt_amd/lib/exp/libpbrt_gpu_tail2.so
PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_tail1.so timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-side-mode > $OUT/bench_B_main.json 2> $OUT/bench_B_main.err || exit 1
echo "B main done"
PBRT_GPU_LIB=$T timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-side-mode > $OUT/bench_B_tail.json 2> $OUT/bench_B_tail.err || exit 1
echo "B tail done"
PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_tail1.so timeout -k 10 300 python tools/heavy_tile.py --tiles 5389 --waves 1,4,8 > $OUT/heavy_main.txt 2>&1 || exit 1
PBRT_GPU_LIB=$T timeout -k 10 300 python tools/heavy_tile.py --tiles 5389 --waves 1,4,8 > $OUT/heavy_tail.txt 2>&1 || exit 1
echo "heavy done"
PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_tail1.so timeout -k 10 300 python tools/shard_sim.py --ns 8 --ranks 0,1,2,3,4,5,6,7 > $OUT/shard8_main.txt 2>&1 || exit 1
PBRT_GPU_LIB=$T timeout -k 10 300 python tools/shard_sim.py --ns 8 --ranks 0,1,2,3,4,5,6,7 > $OUT/shard8_tail.txt 2>&1 || exit 1
echo "shard done"
PBRT_GPU_LIB=$T timeout -k 10 300 python bench.py --config C --steps 1 --no-cpu-baseline --no-side-mode > $OUT/bench_C_tail.json 2> $OUT/bench_C_tail.err || exit 1
PBRT_GPU_LIB=$T timeout -k 10 300 python bench.py --config D --steps 2 --no-cpu-baseline --no-side-mode > $OUT/bench_D_tail.json 2> $OUT/bench_D_tail.err || exit 1
echo "C D tail done"
