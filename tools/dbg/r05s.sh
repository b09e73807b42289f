set -o pipefail
OUT=gpurun_out/r05s; mkdir -p $OUT; export TMPDIR=/tmp
for q in 1 3; do
PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_q8_$q.so timeout -k 10 400 python bench.py --config D --steps 2 --no-cpu-baseline --no-side-mode > $OUT/bench_D_q8_$q.json 2> $OUT/bench_D_q8_$q.err || exit 1
echo "q8=$q done"
done
timeout -k 10 400 python bench.py --config D --steps 2 --no-cpu-baseline --no-side-mode > $OUT/bench_D_q8_2.json 2> $OUT/bench_D_q8_2.err || exit 1
echo "q8=2 done"
