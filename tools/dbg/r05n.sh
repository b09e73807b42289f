set -o pipefail
OUT=gpurun_out/r05n; mkdir -p $OUT; export TMPDIR=/tmp
for q in 1 3 4; do
PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_q$q.so timeout -k 10 400 python bench.py --config D --steps 2 --no-cpu-baseline --no-side-mode > $OUT/bench_D_q$q.json 2> $OUT/bench_D_q$q.err || exit 1
echo "q$q done"
done
