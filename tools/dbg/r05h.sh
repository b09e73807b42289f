set -o pipefail
OUT=gpurun_out/r05h2; mkdir -p $OUT; export TMPDIR=/tmp
for v in new old new2 old2; do
L=""; [[ $v == old* ]] && L=go-pbrt_amd/lib/exp/libpbrt_gpu_old.so
PBRT_GPU_LIB=$L timeout -k 10 200 python bench.py --config H --steps 5 --no-cpu-baseline --no-side-mode > $OUT/bench_H_$v.json 2> $OUT/bench_H_$v.err || exit 1
echo "$v done"
done
