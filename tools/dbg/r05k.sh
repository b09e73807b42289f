set -o pipefail
OUT=gpurun_out/r05k; mkdir -p $OUT; export TMPDIR=/tmp
V=go-pbrt_amd/lib/exp/libpbrt_gpu_filmv3.so
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-side-mode"
SQ1=SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_ACTIVE_INST_VALU
SQ2=SQ_WAIT_INST_LDS,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_INST_CYCLES_VMEM,SQ_ACTIVE_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_THREAD_CYCLES_VALU
PBRT_GPU_LIB=$V timeout -s KILL 120 rocprofv3 --pmc $SQ1 --output-format csv -d $OUT/sq1 -o sq1 -- $B > $OUT/sq1.log 2>&1 && echo "sq1 done" &&
PBRT_GPU_LIB=$V timeout -s KILL 120 rocprofv3 --pmc $SQ2 --output-format csv -d $OUT/sq2 -o sq2 -- $B > $OUT/sq2.log 2>&1 && echo "sq2 done" &&
PBRT_GPU_LIB=$V timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $B > $OUT/fetch.log 2>&1 && echo "fetch done" &&
PBRT_GPU_LIB=$V timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $B > $OUT/write.log 2>&1 && echo "write done"
