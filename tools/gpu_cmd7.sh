# ad-hoc GPU session 7: candidate stride 1 vs 2 on the long-path scenes (G: glass, D: mesh) at N=1
set -o pipefail
O=gpurun_out/r03g; mkdir -p $O
PBRT_CI_STRIDE=1 timeout -k 10 200 python bench.py --config G --steps 2 --no-cpu-baseline --no-side-mode > $O/bench_G_s1.json 2> $O/bench_G_s1.err &&
timeout -k 10 200 python bench.py --config G --steps 2 --no-cpu-baseline --no-side-mode > $O/bench_G_s2.json 2> $O/bench_G_s2.err &&
PBRT_CI_STRIDE=1 timeout -k 10 200 python bench.py --config D --steps 2 --no-cpu-baseline --no-side-mode > $O/bench_D_s1.json 2> $O/bench_D_s1.err &&
PBRT_CI_STRIDE=1 timeout -k 10 300 python bench.py --config C --steps 1 --no-cpu-baseline --no-side-mode > $O/bench_C_s1.json 2> $O/bench_C_s1.err
echo rc=$?
