set -o pipefail
OUT=gpurun_out/r05z2; mkdir -p $OUT; export TMPDIR=/tmp
for k in 0 2 3 4 5; do
PBRT_PATHS_OVERLAP=$k timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline --no-side-mode > $OUT/bench_B_ov$k.json 2> $OUT/bench_B_ov$k.err || exit 1
echo "B ov$k done"
done
