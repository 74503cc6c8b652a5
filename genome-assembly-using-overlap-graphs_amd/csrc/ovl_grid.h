// ovl_grid.h — the resident scoring grid's interface between its kernel (ovl_kernels.hip resident_kernel) and its
// host side (ovl_resident.h).  Kept apart from ovl_kernels.h so that the other kernel files do not depend on it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// The resident scoring grid (ovl_kernels.hip resident_kernel; host side ovl_resident.h).  One request: score
// pairs [0, n_pairs) of a_idx / b_idx (device pointers into the resident candidate list) like uniform_kernel's
// streamed tile records, into a ring of records in pinned host memory: the request's tile t goes to ring tile
// ri = (pos + t) mod 2^ring_log2 with phase bit ((pos + t) >> ring_log2) + 1 (mod 2), so a ring tile's dwords
// from the lap before carry the other phase and the host needs no store into the ring to reuse it; a special
// pair's word is 8 bytes {payload, seq} at sp[64 ri + lane], current when its high half is this request's seq.
struct OvlResidentBody {
    uint64_t seq;               // the request's sequence number (the device copies' seqlock word)
    int64_t n_pairs;
    const int32_t* a_idx;
    const int32_t* b_idx;
    uint32_t* rec;              // ring records, 32 dwords per ring tile (device address of pinned memory)
    uint64_t* sp;               // ring specials, 64 per ring tile
    int64_t pos;                // ring position of the request's tile 0
    int64_t ring_log2;
    int64_t scoring;            // (uint32)match | (uint64)(uint32)mismatch << 32
    const int32_t* heavy_ids;   // heavy tiles first (uniform_kernel's order), or null
    int64_t heavy_n;
    int64_t tile_base;          // the request's first pair / 64 within the candidate list (tile_flags index)
    int64_t fence;              // the ring's memory is cached in the XCD's L2 (fine-grained): records written back
                                // by a release fence -- 2 one per block, by its last wavefront to finish; 1 one per
                                // wavefront, after its last tile; 0: uncached ring memory, no fence
};
constexpr int kResidentBodyWords = (int)(sizeof(OvlResidentBody) / 8);
// The host's mailbox (pinned, fine-grained): the host writes body[seq & 1], then ctl = seq with a release store;
// bit 32 of ctl asks the grid to leave.  Only block 0 reads it; the other blocks learn the request from a forward
// word and a seqlocked copy of the body in device memory (fwd / dslot, written by block 0).
struct OvlResidentCtl {
    uint64_t ctl;
    uint64_t pad[15];
    OvlResidentBody body[2];
};
struct OvlResidentArgs {
    const uint32_t* sfx;
    const uint32_t* pfx;
    const int32_t* len;
    int32_t n_reads;
    int32_t lw;                 // the dominant (maximum) read length, <= 254
    int32_t wmax;               // words of 32 bases per read row (1..8)
    const uint32_t* full;
    const uint8_t* tile_flags;
    const OvlResidentCtl* mailbox;  // device address of the host mailbox
    uint32_t* fwd;              // device word: the request block 0 forwarded (0 none yet, ~0 leave)
    OvlResidentBody* dslot;     // four device copies of request bodies (slot seq & 3)
    uint32_t seq_base;          // the last request already served (the grid serves the next one on)
    uint64_t idle_ticks;        // block 0 leaves after this many wall-clock ticks without a request
    uint64_t* status;           // pinned words the grid writes when it leaves (why, its last request; trace)
    uint32_t poll_sleep;        // the other blocks' pause between polls of the forward word, in ~0.1 us units
    int32_t pipelined;          // tiles software-pipelined in fewer, fatter wavefronts (else one at a time)
    uint64_t* tbuf;             // trace (or null): 4 words per wavefront (knew the request, last tile done, records
                                // written back, request seq), then block 0's clock when it saw the request
    int32_t blocks;
};
constexpr uint32_t kResidentLeave = 0xFFFFFFFFu;
extern "C" hipError_t ovl_launch_resident(const OvlResidentArgs* args, hipStream_t stream);
