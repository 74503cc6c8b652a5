"""Host topology seen by a GPU job: the allowed CPUs, NUMA nodes and their CPUs, the GPU's closest NUMA
node (hipDeviceAttributeHostNumaId), and where pinned host memory lands (move_pages query)."""
import ctypes
import glob
import json
import os


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    val = ctypes.c_int(-1)
    # hipDeviceAttributeHostNumaId = 94 in ROCm 7.2's hip_runtime_api.h enum
    rc = hip.hipDeviceGetAttribute(ctypes.byref(val), 94, 0)
    res = {"gpu0_host_numa_id": val.value, "rc": rc, "allowed_cpus": sorted(os.sched_getaffinity(0))}
    nodes = {}
    for p in sorted(glob.glob("/sys/devices/system/node/node*/cpulist")):
        nodes[p.split("/")[-2]] = open(p).read().strip()
    res["nodes"] = nodes
    res["cpu_now"] = os.sched_getcpu() if hasattr(os, "sched_getcpu") else None
    for p in glob.glob("/sys/class/drm/card*/device/numa_node"):
        res.setdefault("drm_numa", {})[p.split("/")[4]] = open(p).read().strip()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
