# local_alignment parity tests, then the bench's local-alignment timing (traceback vs score only).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/local
timeout -k 10 600 python -u -m pytest tests/test_gpu_local.py tests/test_gpu_assembly.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/local/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/local/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "
import sys, json; sys.path.insert(0, 'genome-assembly-using-overlap-graphs_amd')
import bench
from ovlgraph import OverlapEngine
with OverlapEngine(0) as eng:
    print(json.dumps(bench.local_alignment_timing(eng, reps=10)))
" > gpurun_out/local/timing.json 2> gpurun_out/local/timing.err || { tail -5 gpurun_out/local/timing.err; exit 1; }
cat gpurun_out/local/timing.json
