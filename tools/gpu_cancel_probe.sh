# GPU check of cancellation latency and the exact-mode bench (diagnostic)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/cs
timeout -k 10 60 python -u tools/cancel_probe.py 64 > gpurun_out/cs/probe.log 2>&1 && timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_cancel.py -m gpu > gpurun_out/cs/tests.log 2>&1 && timeout -k 10 150 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cs/bench.log 2>&1 && timeout -k 10 150 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --mode throughput > gpurun_out/cs/bench_tp.log 2>&1; echo rc=$?
