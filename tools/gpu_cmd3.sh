# ad-hoc GPU session 3: config D (mesh, path wavefront) profile on the shipped pipeline, and the
# C / E-shard bench lines
set -o pipefail
bash tools/profile_round.sh r03d_D --config D &&
bash tools/final_round.sh r03d benches
echo rc=$?
