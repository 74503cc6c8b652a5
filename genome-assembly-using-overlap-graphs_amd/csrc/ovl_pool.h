// ovl_pool.h — the host side's CPU share detection (CpuShare) and worker pool (CopyPool): host copies,
// expansion of packed results, pair-list encoding and read preparation split over threads (ovl_api.cpp).
// Host code only; tools/pool_probe.cpp times the pool's per-batch cost on its own.
#pragma once

#include <immintrin.h>
#include <pthread.h>
#include <sched.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

namespace {

// Processes that share this process's CPUs and drive libovl (the reference's joblib workers, experiments.py:537
// n_jobs=-1, or torch.distributed ranks).  Each such process holds one abstract unix socket bound to
// "\0ovl-share-<uid>-<cpu set hash>-<slot>": binding fails while another live process holds the slot and the
// kernel releases it when the holder exits, so nothing is left behind.  The count is refreshed at setup calls
// (context creation, ovl_set_reads, ovl_candidates, ovl_host_pool), never inside a scoring call.
class CpuShare {
  public:
    static constexpr int kSlots = 64;
    static CpuShare& get() {
        static std::mutex mu;
        std::lock_guard<std::mutex> lk(mu);
        static CpuShare* one = nullptr;
        if (!one || one->pid_ != getpid()) {  // a forked child holds no slot of its own yet
            if (one && one->fd_ >= 0) close(one->fd_);  // (the parent's slot stays bound through its own fd)
            one = new CpuShare();
        }
        return *one;
    }
    // CPUs this process may run on: its affinity set, capped by the cgroup quota (cpu.max)
    int cpus() const { return cpus_; }
    int sharers() const { return sharers_.load(std::memory_order_relaxed); }
    // join (once per process) and recount: max(bound slots, LOCAL_WORLD_SIZE), at least 1.  A recount probes
    // 64 slots (~90 us on the box), so setup calls reuse a count younger than 50 ms unless `force`
    int refresh(bool force = false) {
        std::lock_guard<std::mutex> lk(mu_);
        const auto now = std::chrono::steady_clock::now();
        if (!force && fd_ >= 0 && now - last_ < std::chrono::milliseconds(50)) return sharers_.load();
        last_ = now;
        if (fd_ < 0) fd_ = bind_slot(-1);
        int bound = 0;
        for (int i = 0; i < kSlots; ++i)
            if (i == slot_ || slot_held(i)) ++bound;
        int ranks = 1;
        if (const char* e = getenv("LOCAL_WORLD_SIZE")) ranks = std::max(1, atoi(e));
        const int n = std::max(std::max(bound, ranks), 1);
        sharers_.store(n, std::memory_order_relaxed);
        return n;
    }

  private:
    CpuShare() : pid_(getpid()) {
        cpu_set_t set;
        CPU_ZERO(&set);
        int n = 0;
        uint64_t h = 1469598103934665603ull ^ (uint64_t)getuid();
        if (sched_getaffinity(0, sizeof(set), &set) == 0) {
            n = CPU_COUNT(&set);
            for (int c = 0; c < CPU_SETSIZE; ++c)
                if (CPU_ISSET(c, &set)) h = (h ^ (uint64_t)c) * 1099511628211ull;
        }
        if (n <= 0) n = (int)std::max(1u, std::thread::hardware_concurrency());
        long long quota = 0, period = 0;
        if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
            if (fscanf(f, "%lld %lld", &quota, &period) != 2) quota = period = 0;  // "max ..." stays 0
            fclose(f);
        }
        if (quota > 0 && period > 0) n = std::min<int>(n, (int)std::max<long long>(1, quota / period));
        cpus_ = n;
        snprintf(key_, sizeof(key_), "ovl-share-%u-%016llx", (unsigned)getuid(), (unsigned long long)h);
    }
    socklen_t slot_addr(int i, sockaddr_un& a) const {
        memset(&a, 0, sizeof(a));
        a.sun_family = AF_UNIX;
        const int len = snprintf(a.sun_path + 1, sizeof(a.sun_path) - 1, "%s-%d", key_, i);
        return (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + len);
    }
    // bind the first free slot and keep it (returns its fd, or -1)
    int bind_slot(int) {
        for (int i = 0; i < kSlots; ++i) {
            const int fd = socket(AF_UNIX, SOCK_DGRAM | SOCK_CLOEXEC, 0);
            if (fd < 0) return -1;
            sockaddr_un a;
            const socklen_t n = slot_addr(i, a);
            if (bind(fd, reinterpret_cast<sockaddr*>(&a), n) == 0) {
                slot_ = i;
                return fd;
            }
            const int err = errno;
            close(fd);
            if (err != EADDRINUSE) return -1;
        }
        return -1;
    }
    // a live process holds slot i: a datagram socket can connect to it (connect binds nothing, so two
    // processes probing at once never see each other's probes as holders)
    bool slot_held(int i) const {
        const int fd = socket(AF_UNIX, SOCK_DGRAM | SOCK_CLOEXEC, 0);
        if (fd < 0) return false;
        sockaddr_un a;
        const socklen_t n = slot_addr(i, a);
        const bool held = connect(fd, reinterpret_cast<sockaddr*>(&a), n) == 0;
        close(fd);
        return held;
    }
    pid_t pid_;
    int cpus_ = 1;
    int fd_ = -1, slot_ = -1;
    char key_[64];
    std::atomic<int> sharers_{1};
    std::chrono::steady_clock::time_point last_{};
    std::mutex mu_;
};

// Threads of the host pool for `cpus` CPUs shared by `sharers` processes: OVL_POOL_THREADS (or the older
// OVL_HOST_THREADS) when set, else the process's part of the CPUs less one, at most 12, at least 1.  (Round 2,
// three processes on a 16-CPU share: 6 / 8 / 12 threads each 0.156-0.217 / 0.181-0.229 / 0.157-0.162 ms,
// profiles/r02_pool_threads_*.json.  Round 5, one process, per-rank steps at N = 1 / 2 / 4 / 8 of the target list:
// 12 threads 0.138 / 0.089 / 0.060 / 0.045 ms against 15 threads 0.150 / 0.095 / 0.065 / 0.050, same box; streamed
// records (OVL_PACK=2) preferred 15 by 1-7 %, profiles/r05_pool_threads_ab.json.)
int pool_rule(int cpus, int sharers, int env_threads) {
    if (env_threads > 0) return std::min(64, env_threads);
    return std::max(1, std::min(12, cpus / std::max(1, sharers) - 1));
}

int env_pool_threads() {
    for (const char* k : {"OVL_POOL_THREADS", "OVL_HOST_THREADS"})
        if (const char* e = getenv(k)) return std::max(0, atoi(e));
    return 0;
}

// Host copies between pageable caller arrays and the pinned staging rings, and the expansion of packed results,
// split over a pool of worker threads (one thread copies ~10 GB/s; a 16 MB result column is ~1.5 ms alone).  The
// pool is created on first use in each process (a forked joblib worker builds its own) with the threads the
// rule gives one process alone; a call uses the threads the rule gives with the current sharer count, and the
// workers and the caller poll for work only while this process has its CPUs to itself.
//
// A batch is published without a lock: its function, cuts and part count, then one release store of the claim
// word (batch generation << 32 | next part).  Idle workers poll the claim word and take parts by compare-and-swap
// on it, so a part goes to a worker within a cache-line transfer; the swap only succeeds for the current
// generation, so a worker that read a finished batch's word never runs its function.  Workers that polled longer
// than spin_us_ sleep on a condition variable, and the caller wakes them only when some are asleep (spin_us_ is 0,
// so every batch wakes them, only when this process's part of the CPUs is below two).  (Round 4:
// the mutex-and-queue form handed a batch's parts out one lock at a time, ~11 us per batch of 12 parts on the
// box -- a fixed cost per expanded chunk, tools/shard_step_ab.py traces.)
class CopyPool {
  public:
    // threads a call uses now (the calling thread included)
    static int threads() {
        const CpuShare& cs = CpuShare::get();
        return pool_rule(cs.cpus(), cs.sharers(), env_pool_threads());
    }
    static CopyPool& get() {
        static const int registered = pthread_atfork(nullptr, nullptr, &CopyPool::after_fork);
        (void)registered;
        std::lock_guard<std::mutex> lk(get_mutex());
        if (!pool_ || pool_->pid_ != getpid()) pool_ = new CopyPool();  // a forked child starts a fresh pool
        return *pool_;
    }
    // [0, n) cut into parts of >= min_part items (multiples of 64), one per thread a call may use:
    // part i is [b[i], b[i + 1])
    std::vector<size_t> cut(size_t n, size_t min_part) const {
        const size_t use = (size_t)std::min<int>(threads(), (int)workers_ + 1);
        const size_t parts = std::max<size_t>(1, std::min<size_t>(use, n / std::max<size_t>(min_part, 1)));
        std::vector<size_t> b(1, 0);
        if (parts > 1) {
            const size_t step = (n / parts + 63) & ~size_t(63);
            for (size_t i = 1; i < parts && i * step < n; ++i) b.push_back(i * step);
        }
        b.push_back(n);
        return b;
    }
    // f(i, lo, hi) for every part i of `b` (from cut), on the workers and the calling thread (which runs part 0
    // and then claims parts like a worker); `pre`, when given, runs on the calling thread once the batch is
    // published, before its own part (encode_chunk issues the previous chunk there).  A pool call made from
    // inside `pre` or `f` on this thread (the pool is busy with this batch, and call_mu_ is held) runs its parts
    // inline instead of waiting on itself.
    void parallel_parts(const std::vector<size_t>& b, const std::function<void(size_t, size_t, size_t)>& f,
                        const std::function<void()>& pre = nullptr) {
        // poll while this process's part of the CPUs holds its threads (pool_rule sizes them to it): ranks of a
        // multi-GPU job on one node each own their part, and a sleeping worker's wake-up (~5-10 us) would be paid
        // per batch; only a part below two CPUs (many processes on few CPUs) sleeps at once
        const CpuShare& cs = CpuShare::get();
        const int spin = cs.cpus() / std::max(1, cs.sharers()) >= 2 ? spin_cfg_ : 0;
        spin_us_.store(spin, std::memory_order_relaxed);
        const size_t parts = b.size() - 1;
        if (parts <= 1 || in_batch_) {
            if (pre) pre();
            for (size_t i = 0; i < parts; ++i) f(i, b[i], b[i + 1]);
            return;
        }
        std::lock_guard<std::mutex> one_call(call_mu_);  // calls from several host threads take turns
        struct InBatch {
            InBatch() { in_batch_ = true; }
            ~InBatch() { in_batch_ = false; }
        } in_batch;
        f_ = &f;
        b_ = b.data();
        parts_.store(parts, std::memory_order_relaxed);
        pending_.store(parts - 1, std::memory_order_relaxed);
        const uint64_t gen = (claim_.load(std::memory_order_relaxed) >> 32) + 1;
        claim_.store(gen << 32 | 1u, std::memory_order_seq_cst);  // publish; part 0 is the caller's
        if (sleepers_.load(std::memory_order_seq_cst) > 0) {
            { std::lock_guard<std::mutex> lk(mu_); }  // a worker between its check and its wait has reached the wait
            cv_.notify_all();
        }
        if (pre) pre();
        f(0, b[0], b[1]);
        while (take_part(gen)) {
        }
        // the batch's end: polled for a while (the workers finish within microseconds of the caller), then a
        // blocking wait
        if (!spin_until([&] { return pending_.load(std::memory_order_acquire) == 0; }, spin)) {
            std::unique_lock<std::mutex> lk(mu_);
            waiting_ = true;
            done_.wait(lk, [&] { return pending_.load(std::memory_order_acquire) == 0; });
            waiting_ = false;
        }
        f_ = nullptr;
    }
    // f(lo, hi) over [0, n) cut into parts of >= min_part items (multiples of 64)
    void parallel(size_t n, size_t min_part, const std::function<void(size_t, size_t)>& f) {
        parallel_parts(cut(n, min_part), [&f](size_t, size_t lo, size_t hi) { f(lo, hi); });
    }
    // dst[i] = src[i] for [0, bytes)
    void copy(void* dst, const void* src, size_t bytes) {
        parallel(bytes, kMinPart, [=](size_t lo, size_t hi) { memcpy((char*)dst + lo, (const char*)src + lo, hi - lo); });
    }

  private:
    static constexpr size_t kMinPart = size_t(1) << 19;
    static inline CopyPool* pool_ = nullptr;
    static std::mutex& get_mutex() {
        static std::mutex* mu = new std::mutex();
        return *mu;
    }
    // fork() copies only the calling thread: the child drops the parent's pool (its workers do not exist
    // there, and a mutex another thread held at the fork would never be released) and builds its own
    static void after_fork() {
        new (&get_mutex()) std::mutex();
        pool_ = nullptr;
    }
    CopyPool() : pid_(getpid()) {
        // workers for this process alone (sharers 1); calls with more sharers use fewer of them
        const int n = pool_rule(CpuShare::get().cpus(), 1, env_pool_threads());
        spin_us_.store(spin_cfg_, std::memory_order_relaxed);
        for (int i = 0; i + 1 < n; ++i) {
            std::thread t([this] { run(); });
            t.detach();  // lives with the process; never joined at exit
            ++workers_;
        }
    }
    // poll `ready` for up to `us` microseconds
    template <typename F>
    static bool spin_until(F ready, int us) {
        if (ready()) return true;
        if (us <= 0) return false;
        const auto end = std::chrono::steady_clock::now() + std::chrono::microseconds(us);
        for (int i = 1;; ++i) {
            _mm_pause();
            if (ready()) return true;
            if ((i & 31) == 0 && std::chrono::steady_clock::now() > end) return false;
        }
    }
    // claim and run one part of batch `gen`; false when the batch has no unclaimed part (or is not current)
    bool take_part(uint64_t gen) {
        uint64_t c = claim_.load(std::memory_order_acquire);
        for (;;) {
            if ((c >> 32) != gen) return false;
            const size_t i = (size_t)(c & 0xFFFFFFFFu);
            // (a batch published since c was read fails the swap below)
            if (i >= parts_.load(std::memory_order_relaxed)) return false;
            if (claim_.compare_exchange_weak(c, c + 1, std::memory_order_acq_rel, std::memory_order_acquire)) {
                (*f_)(i, b_[i], b_[i + 1]);
                if (pending_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                    std::lock_guard<std::mutex> lk(mu_);  // the caller tests pending_ under mu_: no lost wake-up
                    if (waiting_) done_.notify_all();
                }
                return true;
            }
        }
    }
    // a worker takes parts of each new batch; it polls for the next for spin_us_ after its last part, then
    // sleeps until a batch is published
    void run() {
        uint64_t seen = claim_.load(std::memory_order_acquire) >> 32;
        for (;;) {
            // (seq_cst: ordered after sleepers_'s increment, against the caller's publish-then-count)
            const auto fresh = [&] { return (claim_.load(std::memory_order_seq_cst) >> 32) != seen; };
            if (!spin_until(fresh, spin_us_.load(std::memory_order_relaxed))) {
                std::unique_lock<std::mutex> lk(mu_);
                sleepers_.fetch_add(1, std::memory_order_seq_cst);
                cv_.wait(lk, fresh);
                sleepers_.fetch_sub(1, std::memory_order_relaxed);
            }
            seen = claim_.load(std::memory_order_acquire) >> 32;
            while (take_part(seen)) {
            }
        }
    }
    pid_t pid_;
    int workers_ = 0;
    std::atomic<uint64_t> claim_{0};  // batch generation << 32 | next unclaimed part
    const std::function<void(size_t, size_t, size_t)>* f_ = nullptr;  // the current batch (valid while it runs)
    const size_t* b_ = nullptr;
    std::atomic<size_t> parts_{0};
    std::atomic<size_t> pending_{0};  // parts 1 .. of the current batch not finished yet
    std::atomic<int> sleepers_{0};    // workers asleep on cv_
    bool waiting_ = false;            // the caller sleeps on done_ (guarded by mu_)
    int spin_cfg_ = 100;              // microseconds a worker polls for work after its last part
    static inline thread_local bool in_batch_ = false;  // this thread is inside parallel_parts (nested calls
                                                        // run inline)
    std::atomic<int> spin_us_{100};   // 0 while this process's part of the CPU set is below two CPUs
    std::mutex mu_, call_mu_;
    std::condition_variable cv_, done_;
};

}  // namespace
