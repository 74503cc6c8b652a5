// ovl_graph.cpp — host-side graph stage after scoring: cycle removal of overlapGraphs.py:106-130.
//
// The reference loop (remove_cycles_from_graph):
//     while G has a cycle:  cycle = nx.find_cycle(G, orientation='original')
//                           remove the cycle's weakest edge (min weight, first in cycle order)
// restarts networkx's edge DFS from the first node after every removal, which is quadratic in the
// number of removed edges (hours at 10,000 reads).  This is an exact replay of that loop that does
// not restart:
//
//  * Start nodes.  find_cycle tries start nodes in graph order, skipping nodes already reached
//    ("explored").  A start whose DFS finds no cycle reaches only acyclic, explored territory, and a
//    removal happens beyond it, so every later call replays those starts unchanged: the replay keeps
//    the current start and its explored set.
//  * Rewind instead of restart.  Within the current start, a fresh call repeats the previous call's
//    DFS event for event up to the moment the removed edge was yielded (that edge lies on the active
//    path: the cycle is a suffix of it).  So the DFS state is rewound to that moment through an undo log
//    (iterator advances, first visits, 'seen' insertions), the edge is marked dead, and the DFS goes on.
//  * Settled nodes.  A node that cannot reach any cycle of the current graph (no path to a
//    non-trivial strongly connected component or a self-loop) never closes a cycle and is never on
//    the path when one closes; removals only delete edges, so it stays that way.  An edge into such
//    a node is skipped like an edge into an explored node: the reference's excursion below it
//    appends and later pops path edges whose heads cannot be the next yield's tail (that node
//    reaches them, so they would be on a cycle with it), leaving the path and active set exactly as
//    they are without the excursion.  The settled set is kept exact after every removal (class Sinks:
//    propagation from the sinks over the reverse edges, O(E) over the whole run), so every removal prunes
//    the re-walk after its rewind at once (target point: 38 M DFS yields instead of 86 M with a set
//    recomputed every E/2 yields).
//  * DFS semantics are networkx 3.x edge_dfs + find_cycle for a DiGraph: one out-edge iterator per node,
//    created at its first visit and resumed when the node is pushed again; an edge into an explored
//    node is skipped (its excursion only yields skipped edges); an edge into an active-path node closes
//    the cycle, which starts at the first path edge leaving that node.
//
// Input is the graph in CSR form: nodes in G's node order, each node's out-edges in its adjacency
// (insertion) order, edge weights.  Output is the removed edges (CSR indices) in removal order.
#include <stddef.h>
#include <stdint.h>

#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <vector>

#include "ovl.h"

namespace {

// An array of n trivially-constructible T in anonymous memory aligned to 2 MB and marked for transparent huge
// pages (madvise; a no-op where THP is off): the replay's edge records are read at random, 45-60 MB at the target
// point, so with 4 KB pages nearly every yield is a TLB miss as well as a cache miss.  Falls back to the heap.
template <typename T>
class HugeArray {
  public:
    explicit HugeArray(size_t n) : n_(n) {
        const size_t align = size_t(2) << 20;
        bytes_ = ((n * sizeof(T) + align - 1) / align + 1) * align;
        void* m = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (m == MAP_FAILED) {
            heap_.resize(n);
            p_ = heap_.data();
            return;
        }
        base_ = m;
        p_ = reinterpret_cast<T*>((reinterpret_cast<uintptr_t>(m) + align - 1) & ~(uintptr_t)(align - 1));
        (void)madvise(p_, n * sizeof(T), MADV_HUGEPAGE);
    }
    ~HugeArray() {
        if (base_) munmap(base_, bytes_);
    }
    HugeArray(const HugeArray&) = delete;
    HugeArray& operator=(const HugeArray&) = delete;
    T* data() { return p_; }
    T& operator[](size_t i) { return p_[i]; }

  private:
    size_t n_, bytes_ = 0;
    void* base_ = nullptr;
    T* p_ = nullptr;
    std::vector<T> heap_;
};

// Nodes whose out-edges are final, published as they become so (ovl_remove_cycles_stream): a node that is
// settled (below) or explored (reached by a start whose walk found no cycle) can reach no cycle, so none of its
// out-edges is ever removed.  nodes[0 .. *count) are published with a release store of *count; a consumer on
// another thread reads *count with an acquire load, then those nodes' rows of the caller's alive array.
struct Publish {
    int32_t* nodes = nullptr;
    int64_t* count = nullptr;
    int64_t k = 0;
    void push(int32_t v) {
        if (!nodes) return;
        nodes[k++] = v;
        __atomic_store_n(count, k, __ATOMIC_RELEASE);
    }
};

// The settled set, kept exact after every removal: settled = the nodes that cannot reach a cycle over the
// live edges.  cnt[x] counts x's live out-edges into unsettled nodes, and x is settled iff cnt[x] == 0 (a node
// whose every path ends in a sink), which propagation from the sinks computes exactly: a node left with
// cnt > 0 has a live edge to another such node, so an infinite path, so a cycle ahead.  Removing an edge only
// grows the set: its tail's count drops, and a tail that reaches 0 settles and decrements the counts of its
// live in-edges' tails.  Each edge is decremented at most once (by its removal or by its head settling), so
// the whole run is O(E).  Settling sets done[v].
class Sinks {
  public:
    Sinks(const int64_t* off, const int32_t* head, int32_t n, uint8_t* done, bool on, Publish* pub)
        : head_(head), done_(done), on_(on), pub_(pub) {
        if (!on_) return;
        const int64_t E = off[n];
        tail_.resize((size_t)E);
        roff_.assign((size_t)n + 1, 0);
        for (int32_t v = 0; v < n; ++v)
            for (int64_t e = off[v]; e < off[v + 1]; ++e) {
                tail_[(size_t)e] = v;
                ++roff_[(size_t)head[e] + 1];
            }
        for (int32_t v = 0; v < n; ++v) roff_[(size_t)v + 1] += roff_[(size_t)v];
        rin_.resize((size_t)E);
        std::vector<int64_t> fill(roff_.begin(), roff_.end() - 1);
        for (int64_t e = 0; e < E; ++e) rin_[(size_t)fill[(size_t)head[e]]++] = (int32_t)e;
        cnt_.resize((size_t)n);
        for (int32_t v = 0; v < n; ++v) {
            cnt_[(size_t)v] = (int32_t)(off[v + 1] - off[v]);
            if (cnt_[(size_t)v] == 0) q_.push_back(v);
        }
        drain(nullptr);
    }
    // edge e = (u, v) was just removed (alive[e] = 0 already)
    void removed(int64_t e, const uint8_t* alive) {
        if (!on_) return;
        const int32_t u = tail_[(size_t)e], v = head_[e];
        if (done_[u] || done_[v]) return;  // (an edge into a settled node was no longer counted)
        if (--cnt_[(size_t)u] == 0) {
            q_.push_back(u);
            drain(alive);
        }
    }

  private:
    void drain(const uint8_t* alive) {
        while (!q_.empty()) {
            const int32_t v = q_.back();
            q_.pop_back();
            done_[v] = 1;
            pub_->push(v);
            for (int64_t k = roff_[(size_t)v]; k < roff_[(size_t)v + 1]; ++k) {
                const int32_t e = rin_[(size_t)k];
                if (alive && !alive[e]) continue;
                const int32_t x = tail_[(size_t)e];
                if (done_[x]) continue;
                if (--cnt_[(size_t)x] == 0) q_.push_back(x);
            }
        }
    }
    const int32_t* head_;
    uint8_t* done_;
    bool on_;
    Publish* pub_;
    std::vector<int32_t> tail_, rin_, cnt_, q_;  // edge tails, in-edges by head, counts, settle queue
    std::vector<int64_t> roff_;                  // in-edge rows
};

}  // namespace

namespace {

// WT: the weight type of the edge records, int32_t when every weight fits (12-byte records: the target point's
// 3.75 M edges take 45 MB instead of 60 MB of cache)
template <typename WT>
// (arguments checked by replay below; n_nodes > 0)
int replay_t(const int64_t* off, const int32_t* head, const int64_t* weight, int32_t n_nodes, int64_t* removed,
             int64_t* n_removed, uint8_t* alive_out, Publish& pub) {
    const int64_t n_edges = off[n_nodes];

    // Per edge: the head, the skip delta to the next edge that may still be yielded (0: this one; edges removed
    // or into explored / settled nodes are spliced out), the weight.  A sentinel record ends the array.  Read only
    // to find a node's next live edge after a yield, not by the yield itself (Node below).
    struct Edge {
        int32_t head;
        int32_t skip;
        WT w;
    };
    HugeArray<Edge> ed((size_t)n_edges + 1);
    for (int64_t e = 0; e < n_edges; ++e) ed[(size_t)e] = {head[e], 0, (WT)weight[e]};
    ed[(size_t)n_edges] = {0, 0, 0};
    std::vector<uint8_t> alive_own(alive_out ? 0 : (size_t)n_edges, 1), done(n_nodes, 0);  // done = explored |
                                                                                            // settled (only grow)
    uint8_t* alive = alive_out ? alive_out : alive_own.data();
    if (alive_out) memset(alive_out, 1, (size_t)n_edges);
    // Per node, what a yield touches, in one record (20 bytes: the target point's 50,000 nodes fit a core's L2).
    // The out-edge iterator is held as the edge it yields next: cq, its CSR index, and when `cv` also its head ch
    // and weight cw, so a yield reads no edge record -- the edge array (45 MB at the target point) is read only to
    // find the next live edge after a yield (cv = 0: scan from cq), off the walk's critical path.  "Live" only ever
    // turns false (removal, head explored / settled), so a cached edge whose head is not done is still the next
    // live one, except the removed edge itself (its tail's cache is dropped at the removal).  Also the row's end
    // (so a yield reads no offset either), visited (= seen: both happen at the yield that first reaches it) and on
    // the active path.  A node starts with its row's first edge cached.  The index of the path edge leaving a node
    // (valid while it is active, read only when a cycle closes) is kept apart, in tail_pos.  (Box, alternating
    // builds: row end in the record and tail_pos apart 0.374 -> 0.354 s; 16-byte records with the flags in a byte
    // array 0.383 -> 0.408 s, not kept; profiles/r05_replay_ab.json.)
    struct Node {
        int32_t cq, end, ch;
        WT cw;
        uint8_t visited, active, cv;
    };
    std::vector<Node> nd((size_t)n_nodes);
    std::vector<int32_t> tail_pos((size_t)n_nodes, 0);
    for (int32_t v = 0; v < n_nodes; ++v) {
        Node& x = nd[(size_t)v];
        x = Node{};
        x.cq = (int32_t)off[v];
        x.end = (int32_t)off[v + 1];
        if (off[v] < off[v + 1]) {
            x.ch = head[off[v]];
            x.cw = (WT)weight[off[v]];
        }
        x.cv = 1;
    }
    // One undo-log record per yield: the yielding node and the edge it yielded (index, head, weight: undoing the
    // yield puts that edge back as the node's cached next edge), and, when the yield reached its head for the
    // first time, that head (`first`; -1 otherwise): its first visit and 'seen' insertion happen at that yield
    // (a yielded head becomes the next current node unless the edge closes a cycle, which rewinds past the
    // yield), so one record undoes all three.  Undoing a node's yields restores its cache as of its first visit,
    // so a first visit after an undone one needs no reset.  (Scans that only move past dead edges are not logged.)
    struct Event {
        int32_t node, q, first, h;
        WT w;
    };
    // find_cycle's `edges`: the active path, one record per path edge: the undo-log size just before it was
    // yielded, its weight, CSR index, tail (the node whose iterator yielded it), head, and `link`: the last
    // earlier path edge whose weight is <= this one's (-1: none).  From the path's end, the link chain visits
    // the suffix minima, so the first minimum of the cycle path[i0..] is the last chain entry >= i0.
    struct PathEdge {
        int64_t ckpt;
        int64_t w;
        int32_t q;
        int32_t tail;
        int32_t head;
        int32_t link;
    };
    std::vector<PathEdge> path;
    std::vector<int32_t> seen_list;
    std::vector<Event> log;
    int64_t nrem = 0;

    // OVL_CYCLES_SETTLE=0 (a test knob): no settled-node pruning, only the explored nodes are skipped
    const char* env_settle = getenv("OVL_CYCLES_SETTLE");
    Sinks sinks(off, head, n_nodes, done.data(), !(env_settle && atoi(env_settle) == 0), &pub);

    Edge* E = ed.data();
    Node* N = nd.data();
    const uint8_t* D = done.data();
    // the first live edge at or after q (end if none).  Edges into explored or settled nodes are walked by
    // edge_dfs without any effect on find_cycle, and both sets only grow, so such an edge is spliced out of
    // every later iteration (skip deltas, shared with the removed edges) instead of being yielded.
    auto next_live = [E, D](int64_t q, int64_t end) -> int64_t {
        for (;;) {
            while (E[q].skip) {  // (path halving)
                const int64_t p1 = q + E[q].skip;
                const int64_t p2 = p1 + E[p1].skip;
                E[q].skip = (int32_t)(p2 - q);
                q = p2;
            }
            if (q >= end) return end;
            if (!D[E[q].head]) return q;
            E[q].skip = 1;
        }
    };
    for (int32_t s = 0; s < n_nodes; ++s) {
        if (done[s]) continue;
        log.clear();
        path.clear();
        seen_list.clear();
        // the edge_dfs stack is implicit: s, then the heads of path[0 .. depth) -- every stack entry but s is the
        // head of a path edge, in order, and find_cycle's path also keeps, until the next yield pops them, the
        // edges whose heads the stack has popped (path[depth ..)).  So s is the root of every path.
        int32_t depth = 0;
        // the start node's first visit is never rewound (every rewind target is a later yield's checkpoint)
        N[s].visited = 1;
        N[s].active = 1;
        seen_list.push_back(s);
        for (;;) {
            const int32_t cur = depth ? path[(size_t)depth - 1].head : s;
            Node& c = N[cur];
            const int64_t end = c.end;
            if (!c.cv || (c.cq < end && D[c.ch])) {  // next live edge of cur's iterator from the edge records
                const int64_t q = next_live(c.cq, end);
                c.cq = (int32_t)q;
                if (q < end) {
                    c.ch = E[q].head;
                    c.cw = E[q].w;
                }
                c.cv = 1;
            }
            const int64_t q = c.cq;
            if (q == end) {  // iterator exhausted: pop
                if (depth > 0) {
                    --depth;
                    continue;
                }
                // s popped: no cycle reachable from it, everything seen is explored for the later starts
                for (int32_t v : seen_list)
                    if (!done[v]) {
                        done[v] = 1;
                        pub.push(v);
                    }
                N[s].active = 0;
                break;
            }
            // yield edge q = (cur, h)
            const int64_t mark = (int64_t)log.size();
            const int32_t h = c.ch;
            const WT w = c.cw;
            log.push_back({cur, (int32_t)q, -1, h, w});
            c.cq = (int32_t)(q + 1);
            c.cv = 0;
            __builtin_prefetch(&E[q + 1]);  // (for cur's next yield, after the walk below h returns to it)
            if ((size_t)depth < path.size()) {
                // backtracking: pop the path back to the edge whose head is cur (emptied: active_nodes = {s})
                for (size_t k = (size_t)depth; k < path.size(); ++k) N[path[k].head].active = 0;
                path.resize((size_t)depth);
            }
            int32_t link = (int32_t)path.size() - 1;
            while (link >= 0 && path[(size_t)link].w > (int64_t)w) link = path[(size_t)link].link;
            tail_pos[(size_t)cur] = (int32_t)path.size();
            path.push_back({mark, (int64_t)w, (int32_t)q, cur, h, link});
            Node& hn = N[h];
            if (hn.active) {
                // cycle: the path suffix from the first edge leaving h (the path is simple, so that edge is
                // tail_pos[h]); remove its weakest edge, the first minimum in cycle order
                const int32_t i0 = tail_pos[(size_t)h];
                const PathEdge* pp = path.data();
                int32_t kmin = (int32_t)path.size() - 1;
                while (pp[kmin].link >= i0) kmin = pp[kmin].link;
                const int64_t dead = pp[kmin].q;
                const int32_t tail_of_dead = pp[kmin].tail;
                removed[nrem++] = dead;
                // release store: the streamed dict builder and the component helper read alive[] with acquire
                // loads on other threads (ovl_remove_cycles_stream), and a node found alone in its component
                // relies on removals becoming visible in program order
                __atomic_store_n(&alive[(size_t)dead], (uint8_t)0, __ATOMIC_RELEASE);
                E[dead].skip = 1;
                sinks.removed(dead, alive);
                // rewind the DFS to the moment `dead` was about to be yielded
                const int64_t target = pp[kmin].ckpt;
                while ((int64_t)log.size() > target) {
                    const Event ev = log.back();
                    log.pop_back();
                    Node& x = N[ev.node];
                    x.cq = ev.q;
                    x.ch = ev.h;
                    x.cw = ev.w;
                    x.cv = 1;
                    if (ev.first >= 0) {
                        N[ev.first].visited = 0;
                        seen_list.pop_back();
                    }
                }
                N[tail_of_dead].cv = 0;  // (its cached next edge is now the removed one)
                // heads leaving the path (not the closing edge's: that node is on the surviving path)
                for (size_t k = (size_t)kmin; k + 1 < path.size(); ++k) N[pp[k].head].active = 0;
                path.resize((size_t)kmin);
                depth = kmin;  // (the stack at that moment: s and the surviving path heads)
                continue;
            }
            if (!hn.visited) {  // first visit (and 'seen' insertion) of h, undone with this yield
                hn.visited = 1;
                seen_list.push_back(h);
                log.back().first = h;
            }
            hn.active = 1;
            depth = (int32_t)path.size();
        }
    }
    *n_removed = nrem;
    return OVL_OK;
}

int replay(const int64_t* off, const int32_t* head, const int64_t* weight, int32_t n_nodes, int64_t* removed,
           int64_t* n_removed, uint8_t* alive_out, Publish& pub) {
    if (!n_removed || n_nodes < 0 || (n_nodes > 0 && (!off || !head || !weight))) return OVL_E_ARG;
    *n_removed = 0;
    if (n_nodes == 0) return OVL_OK;
    const int64_t n_edges = off[n_nodes];
    if (off[0] != 0 || n_edges < 0) return OVL_E_ARG;
    for (int32_t v = 0; v < n_nodes; ++v)
        if (off[v + 1] < off[v]) return OVL_E_ARG;
    for (int64_t e = 0; e < n_edges; ++e)
        if (head[e] < 0 || head[e] >= n_nodes) return OVL_E_ARG;
    if (n_edges > 0 && !removed) return OVL_E_ARG;
    if (n_edges >= (int64_t(1) << 31) - 1) return OVL_E_UNSUPPORTED;  // int32 positions and skip deltas
    bool narrow = true;
    for (int64_t e = 0; e < n_edges && narrow; ++e) narrow = weight[e] == (int32_t)weight[e];
    return narrow ? replay_t<int32_t>(off, head, weight, n_nodes, removed, n_removed, alive_out, pub)
                  : replay_t<int64_t>(off, head, weight, n_nodes, removed, n_removed, alive_out, pub);
}

}  // namespace

extern "C" __attribute__((visibility("default"))) int ovl_remove_cycles(const int64_t* off, const int32_t* head,
                                                                      const int64_t* weight, int32_t n_nodes,
                                                                      int64_t* removed, int64_t* n_removed) {
    Publish none;
    return replay(off, head, weight, n_nodes, removed, n_removed, nullptr, none);
}

// The same replay, publishing its progress for a consumer on another thread: alive[e] (n_edges entries, set to
// 1 here, 0 when edge e is removed) and the nodes whose out-edges are final, final_nodes[0 .. *n_final), each
// node once, in the order they become final; *n_final reaches n_nodes before the call returns (Publish).
extern "C" __attribute__((visibility("default"))) int ovl_remove_cycles_stream(
    const int64_t* off, const int32_t* head, const int64_t* weight, int32_t n_nodes, int64_t* removed,
    int64_t* n_removed, uint8_t* alive, int32_t* final_nodes, int64_t* n_final) {
    if (!alive || !final_nodes || !n_final) return OVL_E_ARG;
    __atomic_store_n(n_final, (int64_t)0, __ATOMIC_RELEASE);
    Publish pub;
    pub.nodes = final_nodes;
    pub.count = n_final;
    return replay(off, head, weight, n_nodes, removed, n_removed, alive, pub);
}
