#!/bin/bash
# round 4: baseline on a fresh box -- default bench line (no CPU baseline) and the rocprof kernel stats of it
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04a}
mkdir -p $OUT
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $OUT/bench.json 2> $OUT/bench.err \
  || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
echo "bench ok"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $GRAFT_REPO_ROOT/$OUT/prof_bench.json 2> $GRAFT_REPO_ROOT/$OUT/prof_bench.err \
  || { echo "rocprof failed"; tail -30 $GRAFT_REPO_ROOT/$OUT/prof_bench.err; exit 1; }
echo "prof ok"
