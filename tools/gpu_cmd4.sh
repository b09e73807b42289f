# ad-hoc GPU session 4: exclusive CUs for a shard's heaviest tiles (PBRT_CI_EXCLUSIVE, experiment build),
# then bench lines for C, D and rank 0's 1/8 shard of E
set -o pipefail
O=gpurun_out/r03e; mkdir -p $O
for k in 32 64 128; do PBRT_GPU_LIB=go-pbrt_amd/lib/libpbrt_gpu_excl.so PBRT_CI_EXCLUSIVE=$k timeout -k 10 200 python -u tools/shard_sim.py --ns 8 --ranks 0,5 > $O/shard_sim_B_excl$k.jsonl 2> $O/shard_sim_B_excl$k.err || exit 1; done &&
PBRT_GPU_LIB=go-pbrt_amd/lib/libpbrt_gpu_excl.so PBRT_CI_EXCLUSIVE=64 timeout -k 10 200 python -u tools/shard_sim.py --ns 4 --ranks 0,3 > $O/shard_sim_B_excl64_n4.jsonl 2> $O/shard_sim_B_excl64_n4.err &&
bash tools/final_round.sh r03e benches
echo rc=$?
