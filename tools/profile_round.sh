#!/bin/bash
# Round evidence on one MI355X: bench line, kernel-trace stats, HBM PMC passes.
# Each GPU step has its own time limit; steps are chained with && so the first
# failure ends the script. Outputs under gpurun_out/<tag>/.
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err &&
echo "bench done" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o ks -- $B > $OUT/ks.log 2>&1 &&
echo "kernel trace done" &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o fetch -- $B > $OUT/pmc_fetch.log 2>&1 &&
echo "fetch done" &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o write -- $B > $OUT/pmc_write.log 2>&1 &&
echo "write done"
