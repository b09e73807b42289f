# ad-hoc GPU session 5: the wave-dense closest hit in k_chain_ci (bvh_walk_dense): parity, then A/B
set -o pipefail
O=gpurun_out/r03f; mkdir -p $O
export PBRT_GPU_LIB=go-pbrt_amd/lib/libpbrt_gpu_dense.so
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_materials.py tests/test_gpu_edges.py tests/test_fixtures.py tests/test_ray_counts.py > $O/pytest_dense.log 2>&1 &&
echo tests-ok &&
timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline --no-side-mode > $O/bench_B_dense.json 2> $O/bench_B_dense.err &&
PBRT_CI_DENSE=0 timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline --no-side-mode > $O/bench_B_nodense.json 2> $O/bench_B_nodense.err &&
timeout -k 10 300 python bench.py --config C --steps 1 --no-cpu-baseline --no-side-mode > $O/bench_C_dense.json 2> $O/bench_C_dense.err &&
timeout -k 10 200 python bench.py --config G --steps 2 --no-cpu-baseline --no-side-mode > $O/bench_G_dense.json 2> $O/bench_G_dense.err
echo rc=$?
