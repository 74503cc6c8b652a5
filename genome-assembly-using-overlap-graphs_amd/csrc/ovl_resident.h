// ovl_resident.h — host side of the resident scoring grid (ovl_kernels.hip resident_kernel): one per device of a
// context, launched on the first eligible call and left running, so a call posts a request into pinned memory and
// expands the ring records as they land -- no launch, no completion event.  Host code only,
// included by ovl_api.cpp.
//
// Protocol (ovl_kernels.h OvlResidentCtl / OvlResidentBody):
//  * the host writes body[seq & 1], then ctl = seq (release); the grid's block 0 polls ctl and forwards the request;
//  * the grid writes each tile's record into ring tile (pos + t) mod R with the lap's phase bit, and each special
//    pair's word as {payload, seq}; the host takes a tile once its 32 dwords carry the phase and its special words
//    the seq, so it never stores into memory the grid writes (a host store into a line a running kernel writes was
//    measured to come back with the device's value, ovl_expand.h);
//  * the grid leaves when ctl's bit 32 is set (stop) or after idle_us without a request; a call that finds the
//    grid gone (its launch event complete) with its records incomplete relaunches it, and the new grid serves the
//    pending request (its seq_base is the one before);
//  * every wait is bounded: a call whose records are still incomplete after kCallLimit stops the grid, marks the
//    context's resident path broken and tells the caller to score the call through the launch pipeline instead.
#pragma once

#include <hip/hip_runtime.h>

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "ovl_expand.h"
#include "ovl_grid.h"
#include "ovl_pool.h"

namespace {

// What a grid is launched over: the resident read set and the candidate list's heavy-tile flags, fixed for its life
// (a call over anything else stops it and launches a new one).
struct ResidentReads {
    const uint32_t* sfx = nullptr;
    const uint32_t* pfx = nullptr;
    const int32_t* len = nullptr;
    int32_t n_reads = 0, lw = 0, wmax = 0;
    const uint32_t* full = nullptr;
    const uint8_t* tile_flags = nullptr;
    bool operator==(const ResidentReads& o) const {
        return sfx == o.sfx && pfx == o.pfx && len == o.len && n_reads == o.n_reads && lw == o.lw &&
               wmax == o.wmax && full == o.full && tile_flags == o.tile_flags;
    }
};

struct ResidentCall {
    const int32_t* d_a = nullptr;  // the request's pairs (device pointers into the resident candidate list)
    const int32_t* d_b = nullptr;
    int64_t n = 0;
    const int32_t* heavy_ids = nullptr;  // device heavy tile ids of the request (uniform_kernel's order), or null
    int64_t heavy_n = 0, tile_base = 0;
    int32_t match = 0, mismatch = 0;
    int32_t* out_s = nullptr;  // the caller's arrays (any host memory: the host pool writes them)
    int32_t* out_e = nullptr;
};

// Host memory the grid writes and the host reads (ring, status): fine-grained (coherent), so the grid's stores, once
// written back from the L2 (resident_kernel's release fence), invalidate the lines host threads poll.
constexpr unsigned kRingMem = hipHostMallocPortable | hipHostMallocCoherent;
// The mailbox, which the host writes and the grid's block 0 polls: uncached (MTYPE_UC), so no XCD's L2 serves the
// poll an old copy of the request word (with the coherent kind a polled copy stayed in the L2 for 20 ms and more),
// and, since the grid's reads of it do not snoop the host's caches, the host writes its lines back to memory
// (clflushopt) -- the body before the request word (publish).
constexpr unsigned kMailMem = hipHostMallocPortable | hipHostMallocUncached;

#if !defined(__HIP_DEVICE_COMPILE__)  // (the device pass of a HIP translation unit parses host code too)
__attribute__((target("clflushopt"))) inline void flush_lines_opt(const void* p, size_t n) {
    for (uintptr_t a = (uintptr_t)p & ~uintptr_t(63); a < (uintptr_t)p + n; a += 64) _mm_clflushopt((void*)a);
}
#endif
// write [p, p + n) back from the host's caches to memory (ordered before later stores)
inline void flush_lines(const void* p, size_t n) {
#if !defined(__HIP_DEVICE_COMPILE__)
    static const bool opt = [] {
        __builtin_cpu_init();
        return __builtin_cpu_supports("clflushopt");
    }();
    if (opt) {
        flush_lines_opt(p, n);
    } else {
        for (uintptr_t a = (uintptr_t)p & ~uintptr_t(63); a < (uintptr_t)p + n; a += 64) _mm_clflush((void*)a);
    }
    _mm_sfence();
#else
    (void)p;
    (void)n;
#endif
}

class ResidentGrid {
  public:
    static constexpr int kOk = 0, kFallback = 1, kError = -1;
    // tiles per expansion group (groups go round-robin to the pool's parts); incomplete records a pass skips
    static constexpr int64_t kGroupTiles = 8;
    static constexpr size_t kSkip = 32;

    int32_t device = 0;
    int32_t cu_count = 256;
    int32_t blocks_per_cu = 2;
    int32_t poll_sleep = 4;     // the non-lead blocks' pause between polls (~0.1 us units)
    int32_t pipelined = 1;      // resident_kernel's PF form (tiles software-pipelined) or one tile at a time
    int32_t ring_kind = 0;      // the ring's memory: 0 fine-grained pinned, the records written back by one release
                                // fence per block (the block's last wavefront); 2 the same, one fence per
                                // wavefront; 1 host pages registered uncached for the GPU (MTYPE_UC: nothing kept
                                // in the L2, no fence; the host's own mapping stays cached)
    int64_t idle_us = 20000;     // the grid leaves after this long without a request
    int64_t call_limit_us = 2000000;
    bool broken = false;         // a failed call disabled the resident path of this device
    int64_t n_launches = 0, n_relaunches = 0;
    int64_t last_specials = 0;

    ~ResidentGrid() { release(); }

    bool alive() const { return alive_; }

    // ask the grid to leave and wait for it (bounded by its own deadlines: a block that never saw the request to
    // leave still leaves after 2 x idle_us)
    hipError_t stop() {
        if (!alive_) return hipSuccess;
        hipError_t e = hipSetDevice(device);
        if (e != hipSuccess) return e;
        set_ctl((uint64_t(1) << 32) | seq_);
        e = hipEventSynchronize(ev_);
        alive_ = false;
        set_ctl(seq_);
        unregister();
        return e;
    }

    void release() {
        (void)stop();
        (void)hipSetDevice(device);
        free_ring();
        if (mb_) (void)hipHostFree(mb_);
        if (st_h_) (void)hipHostFree(st_h_);
        st_h_ = nullptr;
        if (tb_h_) (void)hipHostFree(tb_h_);
        tb_h_ = nullptr;
        tb_cap_ = 0;
        if (dev_) (void)hipFree(dev_);
        if (ev_) (void)hipEventDestroy(ev_);
        if (ps_) (void)hipStreamDestroy(ps_);
        rec_h_ = nullptr;
        sp_h_ = nullptr;
        mb_ = nullptr;
        dev_ = nullptr;
        ev_ = nullptr;
        ps_ = nullptr;
        ring_log2_ = -1;
    }

    // Score one request.  kOk: every result is in out_s / out_e (*n_bad bad pairs among them); kFallback: nothing
    // usable was written -- the caller scores the call another way; kError: a HIP error (err).
    int score(const ResidentReads& rd, const ResidentCall& c, int64_t* n_bad, hipError_t* err) {
        *n_bad = 0;
        *err = hipSuccess;
        const int64_t nt = (c.n + 63) / 64;
        if (broken || nt <= 0 || rd.lw <= 0 || rd.lw > 254 || rd.wmax < 1 || rd.wmax > 8) return kFallback;
        hipError_t e = prepare(rd, nt);
        if (busy_) return kFallback;
        if (e != hipSuccess) {
            *err = e;
            return kError;
        }
        const uint32_t s = seq_ + 1;
        OvlResidentBody& b = mb_->body[s & 1];
        b.n_pairs = c.n;
        b.a_idx = c.d_a;
        b.b_idx = c.d_b;
        b.rec = rec_d_;
        b.sp = sp_d_;
        b.pos = pos_;
        b.ring_log2 = ring_log2_;
        b.scoring = (uint64_t)(uint32_t)c.match | (uint64_t)(uint32_t)c.mismatch << 32;
        b.heavy_ids = c.heavy_n > 0 ? c.heavy_ids : nullptr;
        b.heavy_n = c.heavy_n;
        b.tile_base = c.tile_base;
        b.fence = ring_uc_ ? 0 : ring_kind == 2 ? 1 : 2;
        __atomic_store_n(&b.seq, (uint64_t)s, __ATOMIC_RELEASE);
        flush_lines(&b, sizeof(b));
        set_ctl(s);
        const int rc = drain(c, nt, s, n_bad, err);
        if (rc == kOk) {
            seq_ = s;
            pos_ += nt;
            return kOk;
        }
        // the request may still be in the grid: make sure it has left before anything else uses the device
        (void)stop();
        seq_ = s;  // (its records may land later: the next request gets a new sequence number and ring lap)
        pos_ += nt;
        if (!busy_) broken = true;  // (a relaunch that found another thread's grid: only this call falls back)
        return rc;
    }

  private:
    bool alive_ = false;
    hipStream_t ps_ = nullptr;
    hipEvent_t ev_ = nullptr;
    OvlResidentCtl* mb_ = nullptr;        // host mailbox
    OvlResidentCtl* mb_d_ = nullptr;      // ... its device address
    char* dev_ = nullptr;                 // device block: fwd word, then the four body copies
    uint32_t* rec_h_ = nullptr;
    uint32_t* rec_d_ = nullptr;
    uint64_t* sp_h_ = nullptr;
    uint64_t* sp_d_ = nullptr;
    uint64_t* tb_h_ = nullptr;            // the grid's trace (OvlResidentArgs::tbuf), pinned; OVL_TRACE_PIPE only
    int64_t tb_waves_ = 0, tb_cap_ = 0;
    uint64_t* st_h_ = nullptr;            // the grid's exit status (OvlResidentArgs::status), pinned
    uint64_t* st_d_ = nullptr;
    int32_t ring_log2_ = -1;
    int64_t pos_ = 0;
    uint32_t seq_ = 0;
    ResidentReads launched_;

    std::thread::id owner_;  // the thread that launched the grid (the one that drives its context)
    bool busy_ = false;      // the last launch found another thread's grid on the device

    static std::mutex& reg_mu() {
        static std::mutex* m = new std::mutex();
        return *m;
    }
    static std::vector<ResidentGrid*>& reg() {
        static std::vector<ResidentGrid*>* v = new std::vector<ResidentGrid*>();
        return *v;
    }
    void unregister() {
        std::lock_guard<std::mutex> lk(reg_mu());
        auto& v = reg();
        v.erase(std::remove(v.begin(), v.end(), this), v.end());
    }
    // At most one resident grid per device in this process, so no grid waits for CU slots another holds: a grid
    // of another context driven by this thread is stopped (this thread is not inside its call); while another
    // thread's grid is on the device, this context's calls use the launch pipeline (false).
    bool claim_device() {
        const std::thread::id me = std::this_thread::get_id();
        std::vector<ResidentGrid*> mine;
        {
            std::lock_guard<std::mutex> lk(reg_mu());
            for (ResidentGrid* g : reg()) {
                if (g == this || g->device != device) continue;
                if (g->owner_ != me) return false;
                mine.push_back(g);
            }
        }
        for (ResidentGrid* g : mine) (void)g->stop();
        std::lock_guard<std::mutex> lk(reg_mu());
        for (ResidentGrid* g : reg())
            if (g != this && g->device == device) return false;  // (another thread claimed it meanwhile)
        reg().push_back(this);
        owner_ = me;
        return true;
    }

    void set_ctl(uint64_t v) {
        __atomic_store_n(&mb_->ctl, v, __ATOMIC_RELEASE);
        flush_lines(&mb_->ctl, sizeof(uint64_t));
    }

    bool ring_uc_ = false;  // the ring in use is host pages registered uncached (ring_kind 1)
    // a zeroed ring array of `bytes`: fine-grained pinned memory, or (ring_kind 1) 2 MiB-aligned host pages
    // registered for the GPU with MTYPE_UC (hipExtHostRegisterUncached)
    hipError_t ring_alloc(void** h, void** d, size_t bytes) {
        hipError_t e;
        if (ring_kind == 1) {
            const size_t al = size_t(2) << 20, sz = (bytes + al - 1) & ~(al - 1);
            void* p = nullptr;
            if (posix_memalign(&p, al, sz) != 0) return hipErrorOutOfMemory;
            memset(p, 0, sz);
            e = hipHostRegister(p, sz, hipHostRegisterPortable | hipHostRegisterMapped | hipExtHostRegisterUncached);
            if (e != hipSuccess) {
                free(p);
                return e;
            }
            *h = p;
            ring_uc_ = true;
        } else {
            if ((e = hipHostMalloc(h, bytes, kRingMem)) != hipSuccess) return e;
            memset(*h, 0, bytes);
            ring_uc_ = false;
        }
        return hipHostGetDevicePointer(d, *h, 0);
    }
    void ring_free(void* h) {
        if (!h) return;
        if (ring_uc_) {
            (void)hipHostUnregister(h);
            free(h);
        } else {
            (void)hipHostFree(h);
        }
    }
    void free_ring() {
        ring_free(rec_h_);
        ring_free(sp_h_);
        rec_h_ = nullptr;
        sp_h_ = nullptr;
        ring_log2_ = -1;
    }

    static bool trace_on() {
        static const bool on = [] {
            const char* v = getenv("OVL_TRACE_PIPE");
            return v && atoi(v) != 0;
        }();
        return on;
    }
    // OVL_TRACE_PIPE=1: why the grid left (its status words), on stderr
    void trace_exit(const char* what, uint32_t s) const {
        if (!trace_on() || !st_h_) return;
        const volatile uint64_t* st = st_h_;
        fprintf(stderr, "ovl_resident: %s at request %u: block 0 left (1 asked, 2 idle, 3 body) %llu, its last %llu, "
                        "ctl seq %llu, body seq %llu, idle ticks %llu, a block on its own deadline %llu\n",
                what, s, (unsigned long long)st[0], (unsigned long long)st[1], (unsigned long long)(st[2] & 0xFFFFFFFFu),
                (unsigned long long)(st[2] >> 32), (unsigned long long)st[3], (unsigned long long)st[4]);
    }

    hipError_t prepare(const ResidentReads& rd, int64_t nt) {
        hipError_t e = hipSetDevice(device);
        if (e != hipSuccess) return e;
        if (!ps_) {
            if ((e = hipStreamCreateWithFlags(&ps_, hipStreamNonBlocking)) != hipSuccess) return e;
            if ((e = hipEventCreateWithFlags(&ev_, hipEventDisableTiming)) != hipSuccess) return e;
            if ((e = hipHostMalloc((void**)&mb_, sizeof(OvlResidentCtl), kMailMem)) !=
                hipSuccess)
                return e;
            memset(mb_, 0, sizeof(OvlResidentCtl));
            flush_lines(mb_, sizeof(OvlResidentCtl));
            if ((e = hipHostGetDevicePointer((void**)&mb_d_, mb_, 0)) != hipSuccess) return e;
            if ((e = hipMalloc((void**)&dev_, 256 + 4 * sizeof(OvlResidentBody))) != hipSuccess) return e;
            if ((e = hipHostMalloc((void**)&st_h_, 64, kRingMem)) != hipSuccess)
                return e;
            memset(st_h_, 0, 64);
            if ((e = hipHostGetDevicePointer((void**)&st_d_, st_h_, 0)) != hipSuccess) return e;
        }
        // the ring: a power of two of at least the request's tiles; sequence numbers far from wrapping (a fresh ring
        // and numbering: no ring word of an old lap or request can match)
        if ((int64_t(1) << std::max(ring_log2_, 0)) < nt || ring_log2_ < 0 || seq_ >= 0xFFFFFF00u) {
            if ((e = stop()) != hipSuccess) return e;
            int32_t lg = 10;
            while ((int64_t(1) << lg) < nt) ++lg;
            lg = std::max(lg, ring_log2_);
            free_ring();
            const size_t tiles = size_t(1) << lg;
            if ((e = ring_alloc((void**)&rec_h_, (void**)&rec_d_, tiles * 128)) != hipSuccess) return e;
            if ((e = ring_alloc((void**)&sp_h_, (void**)&sp_d_, tiles * 64 * sizeof(uint64_t))) != hipSuccess) return e;
            ring_log2_ = lg;
            pos_ = 0;
            seq_ = 0;
            set_ctl(0);
        }
        if (alive_ && !(launched_ == rd) && (e = stop()) != hipSuccess) return e;
        if (!alive_) return launch(rd);
        return hipSuccess;
    }

    hipError_t launch(const ResidentReads& rd) {
        busy_ = false;
        if (!claim_device()) {
            busy_ = true;
            return hipErrorNotReady;
        }
        hipError_t e = hipMemsetAsync(dev_, 0, 256, ps_);  // fwd = 0: nothing forwarded yet
        if (e != hipSuccess) return e;
        int clk_khz = 100000;
        (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, device);
        OvlResidentArgs a{};
        a.sfx = rd.sfx;
        a.pfx = rd.pfx;
        a.len = rd.len;
        a.n_reads = rd.n_reads;
        a.lw = rd.lw;
        a.wmax = rd.wmax;
        a.full = rd.full;
        a.tile_flags = rd.tile_flags;
        a.mailbox = mb_d_;
        a.fwd = reinterpret_cast<uint32_t*>(dev_);
        a.dslot = reinterpret_cast<OvlResidentBody*>(dev_ + 256);
        a.seq_base = seq_;
        a.idle_ticks = (uint64_t)std::max<int64_t>(1, idle_us) * (uint64_t)clk_khz / 1000u;
        memset(st_h_, 0, 64);  // (no grid runs: the stream's previous one has ended)
        a.status = st_d_;
        a.poll_sleep = (uint32_t)std::max(0, poll_sleep);
        a.pipelined = pipelined;
        a.blocks = std::max(1, cu_count * std::max(1, blocks_per_cu));
        // (trace: 4 words per wavefront of the grid, then block 0's word at 16 * blocks -- sized from the grid
        // launched here, reallocated when a grid has more wavefronts than the buffer holds)
        a.tbuf = nullptr;
        if (trace_on()) {
            const int64_t need = 16 * (int64_t)a.blocks + 8;
            if (tb_cap_ < need) {
                if (tb_h_) (void)hipHostFree(tb_h_);
                tb_h_ = nullptr;
                tb_cap_ = 0;
                if (hipHostMalloc((void**)&tb_h_, (size_t)need * sizeof(uint64_t), kRingMem) == hipSuccess) {
                    memset(tb_h_, 0, (size_t)need * sizeof(uint64_t));
                    tb_cap_ = need;
                }
            }
            if (tb_h_ && hipHostGetDevicePointer((void**)&a.tbuf, tb_h_, 0) != hipSuccess) a.tbuf = nullptr;
            tb_waves_ = 4 * (int64_t)a.blocks;
        }
        if ((e = ovl_launch_resident(&a, ps_)) != hipSuccess) return e;
        if ((e = hipEventRecord(ev_, ps_)) != hipSuccess) return e;
        launched_ = rd;
        alive_ = true;
        ++n_launches;
        return hipSuccess;
    }

    // The host pool expands the request's records as they land: tiles in groups of kGroupTiles round-robin over the
    // parts; a pass takes every complete record of the part's pending tiles (skipping up to kSkip incomplete ones)
    // and polls when it took none.  Part 0 (the calling thread) watches the grid: gone with records missing -> it is
    // relaunched (at most twice per call); past call_limit_us -> the call fails over.
    int drain(const ResidentCall& c, int64_t nt, uint32_t s, int64_t* n_bad, hipError_t* err) {
        const ovl_expand::RecK rk{c.match, c.mismatch};
        static const bool a512 = ovl_expand::rec_avx512();
        const bool al = ((uintptr_t)c.out_s & 63) == 0 && ((uintptr_t)c.out_e & 63) == 0;
        const int64_t mask = (int64_t(1) << ring_log2_) - 1;
        const int lg = ring_log2_;
        const int64_t pos = pos_;
        CopyPool& pool = CopyPool::get();
        const std::vector<size_t> parts = pool.cut(64 * 64, 64);
        const int64_t P = (int64_t)parts.size() - 1;
        const int64_t ngroups = (nt + kGroupTiles - 1) / kGroupTiles;
        std::atomic<int> state{0};  // 0 running, 2 failed
        std::atomic<int64_t> left{nt}, bad{0}, specials{0};
        const auto t0 = std::chrono::steady_clock::now();
        std::atomic<int64_t> t_first{-1};  // (trace: ns from the post to the first record taken, then to the
        std::atomic<int64_t> t_half{-1}, t_90{-1}, t_99{-1};  // moments half, 90 % and 99 % of the tiles were taken)
        int relaunches = 0;
        hipError_t herr = hipSuccess;
        // one check of the call's progress: false ends the part (the call failed).  The calling thread (part 0) also
        // watches the grid and relaunches it when it has left with records missing.
        const auto watch = [&](size_t i) -> bool {
            if (state.load(std::memory_order_relaxed) != 0) return false;
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            if (us > (double)call_limit_us) {
                state.store(2, std::memory_order_relaxed);
                return false;
            }
            if (i != 0) return true;
            const hipError_t q = hipEventQuery(ev_);
            if (q == hipErrorNotReady) return true;
            if (q != hipSuccess) {
                herr = q;
                state.store(2, std::memory_order_relaxed);
                return false;
            }
            // the grid has left (idle, or asked to by another context's launch) before this request's end: a new
            // one serves the pending request (records already taken stay taken: the new grid writes the same values)
            trace_exit("relaunch", s);
            alive_ = false;
            unregister();
            const hipError_t le = ++relaunches <= 2 ? launch(launched_) : hipErrorUnknown;
            ++n_relaunches;
            if (le != hipSuccess) {
                if (relaunches <= 2 && !busy_) herr = le;
                state.store(2, std::memory_order_relaxed);
                return false;
            }
            return true;
        };
        pool.parallel_parts(parts, [&](size_t i, size_t, size_t) {
            std::vector<int64_t> pend;
            pend.reserve((size_t)(nt / P + 2 * kGroupTiles));
            for (int64_t gi = (int64_t)i; gi < ngroups; gi += P)
                for (int64_t t = gi * kGroupTiles, t1 = std::min(nt, (gi + 1) * kGroupTiles); t < t1; ++t)
                    pend.push_back(t);
            int nbad = 0;
            int64_t nsp = 0;
            uint32_t polls = 0;
            while (!pend.empty()) {
                size_t keep = 0, skipped = 0, x = 0, took = 0;
                for (; x < pend.size() && skipped < kSkip; ++x) {
                    const int64_t t = pend[x];
                    const int64_t gpos = pos + t;
                    const int64_t ri = gpos & mask;
                    const uint32_t phase = (uint32_t)((gpos >> lg) + 1) & 1u;
                    const uint32_t* r = rec_h_ + 32 * ri;
                    const ovl_expand::RingSp sp{sp_h_ + 64 * ri, s};
                    const int64_t cnt = std::min<int64_t>(64, c.n - 64 * t);
                    int got;
                    if (a512 && cnt == 64) {
                        bool ready = false;
                        got = ovl_expand::rec_tile_avx512_t(c.out_s + 64 * t, c.out_e + 64 * t, r, rk, phase, al,
                                                            &ready, &nbad, sp);
                        if (!ready) got = -2;
                    } else {
                        got = ovl_expand::rec_tile_scalar_t(c.out_s + 64 * t, c.out_e + 64 * t, r, rk, (size_t)cnt,
                                                            phase, &nbad, sp);
                    }
                    if (got >= 0) {
                        nsp += got;
                        ++took;
                    } else {
                        pend[keep++] = t;
                        ++skipped;
                    }
                }
                for (; x < pend.size(); ++x) pend[keep++] = pend[x];
                pend.resize(keep);
                if (took) {
                    if (trace_on() && t_first.load(std::memory_order_relaxed) < 0) {
                        int64_t none = -1;
                        t_first.compare_exchange_strong(
                            none, (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                      std::chrono::steady_clock::now() - t0).count());
                    }
                    const int64_t was = left.fetch_sub((int64_t)took, std::memory_order_relaxed);
                    if (trace_on()) {
                        const int64_t now = (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                                std::chrono::steady_clock::now() - t0).count();
                        const int64_t after = was - (int64_t)took;
                        if (was > nt / 2 && after <= nt / 2) t_half.store(now);
                        if (was > nt / 10 && after <= nt / 10) t_90.store(now);
                        if (was > nt / 100 && after <= nt / 100) t_99.store(now);
                    }
                    polls = 0;
                    continue;
                }
                if (pend.empty()) break;
                _mm_pause();
                if ((++polls & 255) == 0 && !watch(i)) break;
            }
            // (the calling thread keeps watching the grid until every part's tiles are in)
            while (i == 0 && left.load(std::memory_order_relaxed) > 0) {
                _mm_pause();
                if ((++polls & 255) == 0 && !watch(i)) break;
            }
            bad.fetch_add(nbad, std::memory_order_relaxed);
            specials.fetch_add(nsp, std::memory_order_relaxed);
            _mm_sfence();  // (this part's non-temporal stores drained before the part is reported done)
        });
        _mm_sfence();
        if (trace_on() && tb_h_) {  // the grid's side of this request (wall clock, 100 MHz), from block 0's sight of it
            const volatile uint64_t* t = tb_h_;
            const uint64_t t0g = t[4 * tb_waves_];
            std::vector<double> seen, done, wb;
            for (int64_t w = 0; w < tb_waves_; ++w) {
                if (t[4 * w + 3] != s) continue;
                seen.push_back((double)(int64_t)(t[4 * w] - t0g) * 0.01);
                done.push_back((double)(int64_t)(t[4 * w + 1] - t0g) * 0.01);
                wb.push_back((double)(int64_t)(t[4 * w + 2] - t[4 * w + 1]) * 0.01);
            }
            const auto pct = [](std::vector<double>& v, double f) {
                if (v.empty()) return -1.0;
                std::sort(v.begin(), v.end());
                return v[(size_t)(f * (double)(v.size() - 1))];
            };
            fprintf(stderr, "ovl_resident: grid side of request %u (%zu wavefronts with tiles; us after block 0 saw it): "
                            "knew it median %.2f max %.2f; last tile done median %.2f p90 %.2f max %.2f; write-back "
                            "median %.2f max %.2f\n",
                    s, seen.size(), pct(seen, 0.5), pct(seen, 1.0), pct(done, 0.5), pct(done, 0.9), pct(done, 1.0),
                    pct(wb, 0.5), pct(wb, 1.0));
        }
        if (trace_on())
            fprintf(stderr, "ovl_resident: request %u, %lld tiles: first record taken %.1f us after the post, half %.1f, "
                            "90%% %.1f, 99%% %.1f, all %.1f us\n",
                    s, (long long)nt, (double)t_first.load() * 1e-3, (double)t_half.load() * 1e-3,
                    (double)t_90.load() * 1e-3, (double)t_99.load() * 1e-3,
                    std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        *n_bad = bad.load();
        last_specials = specials.load();
        if (state.load() != 0) {
            *err = herr;
            return herr != hipSuccess ? kError : kFallback;
        }
        return kOk;
    }
};

}  // namespace
