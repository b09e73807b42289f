set -o pipefail
OUT=gpurun_out/r05v; mkdir -p $OUT; export TMPDIR=/tmp
T=go-pbrt_amd/lib/exp/libpbrt_gpu_tail2.so
PBRT_GPU_LIB=$T timeout -k 10 150 python bench.py --steps 3 --no-cpu-baseline --no-side-mode > $OUT/bench_B_tail2.json 2> $OUT/bench_B_tail2.err || exit 1
echo "B tail2 done"
PBRT_GPU_LIB=$T timeout -k 10 150 python tools/heavy_tile.py --tiles 5389 --waves 1,4,8 > $OUT/heavy_tail2.txt 2>&1 || exit 1
echo "heavy done"
PBRT_GPU_LIB=$T timeout -k 10 150 python tools/shard_sim.py --ns 8 --ranks 0,1,2,3,4,5,6,7 > $OUT/shard8_tail2.txt 2>&1 || exit 1
echo "shard done"
PBRT_GPU_LIB=$T timeout -k 10 170 python bench.py --config C --steps 1 --no-cpu-baseline --no-side-mode > $OUT/bench_C_tail2.json 2> $OUT/bench_C_tail2.err || exit 1
echo "C done"
