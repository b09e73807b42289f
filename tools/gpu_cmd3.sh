# ad-hoc GPU session 3: where a config-B chain step goes (steptime / diag builds, tools/phase_stats.py),
# then the config-D profile on the shipped pipeline (path wavefront)
set -o pipefail
O=gpurun_out/r03d; mkdir -p $O
PBRT_GPU_LIB=go-pbrt_amd/lib/libpbrt_gpu_steptime.so timeout -k 10 200 python -u tools/phase_stats.py > $O/phase_steptime_B.txt 2>&1 &&
PBRT_GPU_LIB=go-pbrt_amd/lib/libpbrt_gpu_diag.so timeout -k 10 200 python -u tools/phase_stats.py > $O/phase_diag_B.txt 2>&1 &&
bash tools/profile_round.sh r03d_D --config D
echo rc=$?
