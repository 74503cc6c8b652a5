# packed step: bench.py's Workload timed as bench.py times it vs fresh arrays (tools/bench_step_probe.py),
# host pool at 8 (default), 4 and 16 threads
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pk
timeout -k 10 300 python tools/bench_step_probe.py 50 > gpurun_out/pk/bprobe.json && cat gpurun_out/pk/bprobe.json && \
OVL_HOST_THREADS=4 timeout -k 10 300 python tools/bench_step_probe.py 50 > gpurun_out/pk/bprobe_t4.json && cat gpurun_out/pk/bprobe_t4.json && \
OVL_HOST_THREADS=16 timeout -k 10 300 python tools/bench_step_probe.py 50 > gpurun_out/pk/bprobe_t16.json && cat gpurun_out/pk/bprobe_t16.json && \
nproc && numactl --show 2>/dev/null | head -5; lscpu | grep -i "numa\|model name\|socket" | head -8; cat /sys/class/drm/card*/device/numa_node 2>/dev/null | head -10 | tr '\n' ' '
