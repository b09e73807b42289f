# ad-hoc GPU session: kX material tests + benches + occupancy variants + full suite (each GPU step under its own limit)
set -o pipefail
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_materials.py > $O/pytest_mat.log 2>&1 &&
echo mat-ok &&
timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline --no-side-mode > $O/bench_B.json 2> $O/bench_B.err &&
for v in v3 v4; do PBRT_GPU_LIB=go-pbrt_amd/lib/libpbrt_gpu_$v.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side-mode > $O/bench_B_$v.json 2> $O/bench_B_$v.err || exit 1; done &&
timeout -k 10 300 python bench.py --config G --steps 2 --no-cpu-baseline > $O/bench_G.json 2> $O/bench_G.err &&
PBRT_PATHS_WF=1 timeout -k 10 300 python bench.py --config G --steps 2 --no-cpu-baseline --no-side-mode > $O/bench_G_pw.json 2> $O/bench_G_pw.err &&
PBRT_PATHS_WF=1 PBRT_PW_SORT=1 timeout -k 10 300 python bench.py --config G --steps 2 --no-cpu-baseline --no-side-mode > $O/bench_G_pw_sort.json 2> $O/bench_G_pw_sort.err &&
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests --deselect tests/test_materials.py > $O/pytest_all.log 2>&1
echo rc=$?
