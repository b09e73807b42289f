#!/bin/bash
# One GPU session on the MI355X box: the named steps in order, each under its own
# time limit, chained so that the first failure ends the session. Outputs land in
# gpurun_out/<tag>/ (merged back by gpurun).
#   tools/gpu_session.sh <tag> <step> [<step> ...]
# steps:
#   tests                 the whole GPU suite
#   tests=<expr>          GPU tests selected with pytest -k <expr> (commas read as spaces: a,or,b)
#   bench=<cfg>[,args]    bench.py --config <cfg> (no CPU baseline, no side mode);
#                         extra bench args after commas, e.g. bench=C,--steps,1
#   benchfull=<cfg>       bench.py --config <cfg> with its CPU baseline and side mode
#   profile=<cfg>         tools/profile_round.sh for that config
#   phase=<diag|steptime> tools/phase_stats.py with lib/exp/libpbrt_gpu_<build>.so (config B)
#   libbench=<v>,<cfg>    bench.py --config <cfg> --steps 2 with lib/exp/libpbrt_gpu_<v>.so (experiment builds)
#   envbench=VAR=V[+VAR2=V2],<cfg>[,args]  bench.py --config <cfg> with those environment variables
#   py=<script>[~args]    python tools/<script>.py <args> ('~' between args; output under <tag>/)
#   libpy=<v>,<script>[~args]  py= with lib/exp/libpbrt_gpu_<v>.so (diag / experiment builds)
#   smoke                 __graft_entry__.smoke()
set -o pipefail
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for step in "$@"; do
  case "$step" in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest.log; exit 1; } ;;
  tests=*)
    timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "$(echo "${step#tests=}" | tr ',' ' ')" > $OUT/pytest_k.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest_k.log; exit 1; } ;;
  bench=*)
    spec=${step#bench=}; cfg=${spec%%,*}; extra=""
    [[ "$spec" == *,* ]] && extra=$(echo "${spec#*,}" | tr ',' ' ')
    timeout -k 10 500 python bench.py --config $cfg --no-cpu-baseline --no-side-mode --no-rpc $extra > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || { echo "bench $cfg failed"; tail -20 $OUT/bench_$cfg.err; exit 1; } ;;
  benchfull=*)
    cfg=${step#benchfull=}
    timeout -k 10 600 python bench.py --config $cfg > $OUT/benchfull_$cfg.json 2> $OUT/benchfull_$cfg.err || { echo "bench $cfg failed"; tail -20 $OUT/benchfull_$cfg.err; exit 1; } ;;
  profile=*)
    cfg=${step#profile=}
    bash tools/profile_round.sh ${TAG}/prof_$cfg --config $cfg || { echo "profile $cfg failed"; exit 1; } ;;
  phase=*)   # phase=diag | phase=steptime[,scene]: tools/phase_stats.py on that diagnostics build
    spec=${step#phase=}; lib=${spec%%,*}; scn=readme
    [[ "$spec" == *,* ]] && scn=${spec#*,}
    PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_$lib.so timeout -k 10 300 python tools/phase_stats.py --scene $scn > $OUT/phase_${lib}_$scn.txt 2>&1 || { echo "phase $lib failed"; tail -20 $OUT/phase_${lib}_$scn.txt; exit 1; } ;;
  libbench=*)   # libbench=<variant>,<cfg>: bench.py --config <cfg> with lib/exp/libpbrt_gpu_<variant>.so
    spec=${step#libbench=}; v=${spec%%,*}; cfg=${spec#*,}
    PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_$v.so timeout -k 10 400 python bench.py --config $cfg --no-cpu-baseline --no-side-mode --no-rpc --steps 2 > $OUT/bench_${cfg}_$v.json 2> $OUT/bench_${cfg}_$v.err || { echo "bench $cfg $v failed"; tail -20 $OUT/bench_${cfg}_$v.err; exit 1; } ;;
  envbench=*)   # envbench=VAR=VALUE,<cfg>[,args]: bench.py --config <cfg> (no CPU baseline / side mode) with VAR=VALUE
    spec=${step#envbench=}; kv=${spec%%,*}; rest=${spec#*,}; cfg=${rest%%,*}; extra=""
    [[ "$rest" == *,* ]] && extra=$(echo "${rest#*,}" | tr ',' ' ')
    env $(echo "$kv" | tr '+' ' ') timeout -k 10 500 python bench.py --config $cfg --no-cpu-baseline --no-side-mode --no-rpc $extra > $OUT/bench_${cfg}_${kv}.json 2> $OUT/bench_${cfg}_${kv}.err || { echo "bench $cfg $kv failed"; tail -20 $OUT/bench_${cfg}_${kv}.err; exit 1; } ;;
  py=*)   # py=<tools script>[~args]: python tools/<script>.py args ('~' separates; commas stay), output to <script>_<args>.txt
    spec=${step#py=}; scr=${spec%%~*}; args=""
    [[ "$spec" == *~* ]] && args=$(echo "${spec#*~}" | tr '~' ' ')
    tagf=$(echo "$scr $args" | tr -c 'A-Za-z0-9=.\n-' '_')
    timeout -k 10 400 python tools/$scr.py $args > $OUT/$tagf.txt 2>&1 || { echo "py $scr failed"; tail -20 $OUT/$tagf.txt; exit 1; } ;;
  libpy=*)   # libpy=<variant>,<script>[~args]: as py= with lib/exp/libpbrt_gpu_<variant>.so
    spec=${step#libpy=}; v=${spec%%,*}; spec=${spec#*,}; scr=${spec%%~*}; args=""
    [[ "$spec" == *~* ]] && args=$(echo "${spec#*~}" | tr '~' ' ')
    tagf=$(echo "$v $scr $args" | tr -c 'A-Za-z0-9=.\n-' '_')
    PBRT_GPU_LIB=go-pbrt_amd/lib/exp/libpbrt_gpu_$v.so timeout -k 10 400 python tools/$scr.py $args > $OUT/$tagf.txt 2>&1 || { echo "libpy $scr failed"; tail -20 $OUT/$tagf.txt; exit 1; } ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; } ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "$step done"
done
