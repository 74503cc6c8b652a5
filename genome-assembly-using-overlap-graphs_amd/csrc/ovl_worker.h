// ovl_worker.h -- a host thread per device of a multi-device context (ovl_api.cpp run_pipeline), bound to the CPUs
// of its GPU's NUMA node.  Host code only.
#pragma once

#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>

#include <cctype>
#include <condition_variable>
#include <cstdio>
#include <functional>
#include <mutex>
#include <thread>

// A host thread per device of a multi-device context (run_pipeline): it runs the device's job of each call, on the
// CPUs of the GPU's NUMA node when the process may use them, so N devices' launches, polls and synchronisations run
// side by side instead of one after another on the calling thread.
class DevWorker {
  public:
    explicit DevWorker(int device) : th_([this, device] { run(device); }) {}
    ~DevWorker() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            quit_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    void post(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            task_ = std::move(f);
        }
        cv_.notify_all();
    }

  private:
    // the GPU's NUMA node's CPUs (sysfs), intersected with the process's affinity; unchanged when unknown
    static void bind(int device) {
        char bus[64] = {0};
        if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return;
        for (char* q = bus; *q; ++q) *q = (char)tolower(*q);
        char path[160];
        snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
        int node = -1;
        if (FILE* f = fopen(path, "r")) {
            if (fscanf(f, "%d", &node) != 1) node = -1;
            fclose(f);
        }
        if (node < 0) return;
        snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
        FILE* f = fopen(path, "r");
        if (!f) return;
        cpu_set_t want, have;
        CPU_ZERO(&want);
        int lo, hi;
        char sep;
        while (fscanf(f, "%d", &lo) == 1) {
            hi = lo;
            if (fscanf(f, "%c", &sep) == 1 && sep == '-') {
                if (fscanf(f, "%d", &hi) != 1) break;
                if (fscanf(f, "%c", &sep) != 1) sep = 0;
            }
            for (int cpu = lo; cpu <= hi && cpu < CPU_SETSIZE; ++cpu) CPU_SET(cpu, &want);
            if (sep != ',') break;
        }
        fclose(f);
        if (sched_getaffinity(0, sizeof(have), &have) != 0) return;
        CPU_AND(&want, &want, &have);
        if (CPU_COUNT(&want) > 0) (void)pthread_setaffinity_np(pthread_self(), sizeof(want), &want);
    }
    void run(int device) {
        bind(device);
        (void)hipSetDevice(device);
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return quit_ || task_; });
                if (quit_ && !task_) return;
                f = std::move(task_);
                task_ = nullptr;
            }
            f();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::function<void()> task_;
    bool quit_ = false;
    std::thread th_;
};
