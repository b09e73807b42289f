# GPU session 6: the final build's evidence -- the GPU test suite, the config-B profile (bench line
# with the CPU baseline, kernel trace, HBM and SQ passes), the exclusive-CU shard experiment, then
# bench lines for C and D
set -o pipefail
O=gpurun_out/r03e; mkdir -p $O
bash tools/final_round.sh r03_final tests &&
bash tools/profile_round.sh r03_final_B &&
for k in 32 128; do PBRT_GPU_LIB=go-pbrt_amd/lib/libpbrt_gpu_excl.so PBRT_CI_EXCLUSIVE=$k timeout -k 10 120 python -u tools/shard_sim.py --ns 8 --ranks 0,5 > $O/shard_sim_B_excl$k.jsonl 2> $O/shard_sim_B_excl$k.err || exit 1; done &&
timeout -k 10 300 python bench.py --config C --steps 1 > $O/bench_C.json 2> $O/bench_C.err &&
timeout -k 10 300 python bench.py --config D --steps 2 > $O/bench_D.json 2> $O/bench_D.err
echo rc=$?
