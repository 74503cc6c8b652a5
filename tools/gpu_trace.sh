# Per-wavefront trace of one cfg2 launch (make trace build).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/trace
OVL_LIB_PATH=$GRAFT_REPO_ROOT/genome-assembly-using-overlap-graphs_amd/build/trace/libovl.so timeout -k 10 200 python tools/trace_waves.py ${1:-cfg2} > gpurun_out/trace/${1:-cfg2}.txt 2> gpurun_out/trace/err.txt || { tail -5 gpurun_out/trace/err.txt; exit 1; }
cat gpurun_out/trace/${1:-cfg2}.txt
