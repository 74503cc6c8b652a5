set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== smoke"; timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== pytest gpu"; timeout -k 10 700 python -m pytest tests/ -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== bench"; timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench1.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench1.log
exit $rc
