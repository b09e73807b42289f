set -o pipefail
OUT=gpurun_out/r05ov2; mkdir -p $OUT; export TMPDIR=/tmp
V=go-pbrt_amd/lib/exp/libpbrt_gpu_ovp.so
for t in 100 50 200 100b 0; do
tt=${t%b}
PBRT_GPU_LIB=$V PBRT_PATHS_OVERLAP=$tt timeout -k 10 200 python bench.py --steps 4 --no-cpu-baseline --no-side-mode > $OUT/bench_B_ov$t.json 2> $OUT/bench_B_ov$t.err || exit 1
echo "ov$t done"
done
