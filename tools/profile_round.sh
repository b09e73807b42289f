#!/bin/bash
# Round evidence on one MI355X: bench line, kernel-trace stats, HBM PMC passes
# and two SQ (instruction-mix / utilisation) passes, each a run of its own.
# Each GPU step has its own time limit; steps are chained with && so the first
# failure ends the script. Outputs under gpurun_out/<tag>/.
#   tools/profile_round.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-r01}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-side-mode --no-rpc $*"
SQ1=SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_ACTIVE_INST_VALU
SQ2=SQ_THREAD_CYCLES_VALU,SQ_WAIT_INST_ANY,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_TRANS_F64,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY
timeout -k 10 400 python3 bench.py $* > $OUT/bench.json 2> $OUT/bench.err &&
echo "bench done" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o ks -- $B > $OUT/ks.log 2>&1 &&
echo "kernel trace done" &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o fetch -- $B > $OUT/pmc_fetch.log 2>&1 &&
echo "fetch done" &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o write -- $B > $OUT/pmc_write.log 2>&1 &&
echo "write done" &&
timeout -k 10 300 rocprofv3 --pmc $SQ1 --output-format csv -d $OUT/pmc_sq1 -o sq1 -- $B > $OUT/pmc_sq1.log 2>&1 &&
echo "sq1 done" &&
timeout -k 10 300 rocprofv3 --pmc $SQ2 --output-format csv -d $OUT/pmc_sq2 -o sq2 -- $B > $OUT/pmc_sq2.log 2>&1 &&
echo "sq2 done"
