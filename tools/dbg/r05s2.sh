set -o pipefail
OUT=gpurun_out/r05s2; mkdir -p $OUT; export TMPDIR=/tmp
V=go-pbrt_amd/lib/exp/libpbrt_gpu_ovs.so
PBRT_GPU_LIB=$V timeout -k 10 300 python tools/shard_sim.py --ns 2,4 --ranks 0,1,2,3 > $OUT/shard_ovs.txt 2>&1 || exit 1
echo "ovs done"
PBRT_GPU_LIB=$V timeout -k 10 300 python tools/shard_sim.py --ns 2,4 --ranks 0,1,2,3 --env PBRT_PATHS_OVERLAP=0 > $OUT/shard_noov.txt 2>&1 || exit 1
echo "noov done"
PBRT_GPU_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "split" > $OUT/pytest_split.log 2>&1 || { echo "tests failed"; tail -20 $OUT/pytest_split.log; exit 1; }
echo "tests done"
