set -o pipefail
OUT=gpurun_out/r05p; mkdir -p $OUT; export TMPDIR=/tmp
PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_meshcount.so timeout -k 10 300 python tools/count_mesh_bytes.py > $OUT/meshbytes_wide.json 2> $OUT/meshbytes_wide.err || exit 1
echo "count wide done"
PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_meshcount_bin.so timeout -k 10 300 python tools/count_mesh_bytes.py > $OUT/meshbytes_bin.json 2> $OUT/meshbytes_bin.err || exit 1
echo "count bin done"
PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_wideb.so timeout -k 10 400 python bench.py --config D --steps 2 --no-cpu-baseline --no-side-mode > $OUT/bench_D_wideb.json 2> $OUT/bench_D_wideb.err || exit 1
echo "D wideb done"
