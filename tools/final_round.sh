#!/bin/bash
# Round-end evidence on one MI355X, each GPU step under its own time limit.
#   tools/final_round.sh <tag> tests    the GPU test suite
#   tools/final_round.sh <tag> profile  config-B profile (tools/profile_round.sh)
#   tools/final_round.sh <tag> benches  bench lines for C, D and rank 0's 1/8 shard of E
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
case "$2" in
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 &&
  echo "tests done" ;;
profile)
  bash tools/profile_round.sh ${TAG}_B ;;
benches)
  timeout -k 10 300 python bench.py --config C --steps 1 > $OUT/bench_C.json 2> $OUT/bench_C.err &&
  echo "C done" &&
  timeout -k 10 300 python bench.py --config D --steps 2 > $OUT/bench_D.json 2> $OUT/bench_D.err &&
  echo "D done" &&
  timeout -k 10 500 python bench.py --config E --shard 0/8 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_E.json 2> $OUT/bench_E.err &&
  echo "E done" ;;
*) echo "usage: $0 <tag> tests|profile|benches"; exit 2 ;;
esac
