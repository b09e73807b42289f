# ad-hoc GPU session 2: multi-GPU shard projection (one GPU renders rank r's share) at 4 and 8
# waves per tile, then the config-B rocprofv3 evidence (tools/profile_round.sh)
set -o pipefail
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 400 python -u tools/shard_sim.py --ns 1,2,4 --ranks 0,-1 > $O/shard_sim_B_n124.jsonl 2> $O/shard_sim_B_n124.err &&
timeout -k 10 400 python -u tools/shard_sim.py --ns 8 --ranks 0,1,2,3,4,5,6,7 > $O/shard_sim_B.jsonl 2> $O/shard_sim_B.err &&
PBRT_CI_WAVES=8 timeout -k 10 200 python -u tools/shard_sim.py --ns 4,8 --ranks 0,-1 > $O/shard_sim_B_w8.jsonl 2> $O/shard_sim_B_w8.err &&
timeout -k 10 200 python -u tools/shard_sim.py --ns 8 --ranks 0 --mode throughput > $O/shard_sim_B_tp.jsonl 2> $O/shard_sim_B_tp.err &&
PBRT_GPU_LIB=go-pbrt_amd/lib/libpbrt_gpu_r8.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side-mode > $O/bench_B_r8.json 2> $O/bench_B_r8.err &&
bash tools/profile_round.sh r03c_B
echo rc=$?
