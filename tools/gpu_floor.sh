# Floors for the cfg2 launch (tools/microbench.hip, prebuilt) + a quick cfg2 bench line.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/floor
timeout -k 10 120 genome-assembly-using-overlap-graphs_amd/build/microbench > gpurun_out/floor/microbench.txt 2>&1 || exit 1
cat gpurun_out/floor/microbench.txt
timeout -k 10 300 python bench.py --steps 2000 --warmup 20 --no-extra --no-cpu-baseline > gpurun_out/floor/cfg2.json 2> gpurun_out/floor/cfg2.err || { tail -5 gpurun_out/floor/cfg2.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/floor/cfg2.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_ms'], d['host_buffers'])"
