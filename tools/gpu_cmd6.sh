# GPU session 6: the final build's evidence -- the GPU test suite, then the config-B profile
# (bench line with the CPU baseline, kernel trace, HBM and SQ passes)
set -o pipefail
bash tools/final_round.sh r03_final2 tests &&
bash tools/profile_round.sh r03_final2_B
echo rc=$?
