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
//  * DFS semantics are networkx 3.x edge_dfs + find_cycle for a DiGraph: one out-edge iterator per node,
//    created at its first visit and resumed when the node is pushed again; an edge into an explored
//    node is skipped (its excursion only yields skipped edges); an edge into an active-path node closes
//    the cycle, which starts at the first path edge leaving that node.
//
// Input is the graph in CSR form: nodes in G's node order, each node's out-edges in its adjacency
// (insertion) order, edge weights.  Output is the removed edges (CSR indices) in removal order.
#include <stdint.h>

#include <vector>

#include "ovl.h"

namespace {

struct Event {
    int32_t kind;   // 0: first visit of node, 1: iterator advance (old position), 2: 'seen' insertion
    int32_t node;
    int64_t old;
};

}  // namespace

extern "C" __attribute__((visibility("default"))) int ovl_remove_cycles(const int64_t* off, const int32_t* head,
                                                                      const int64_t* weight, int32_t n_nodes,
                                                                      int64_t* removed, int64_t* n_removed) {
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

    std::vector<uint8_t> alive(n_edges, 1), explored(n_nodes, 0), visited(n_nodes, 0), active(n_nodes, 0),
        seen(n_nodes, 0);
    std::vector<int64_t> pos(n_nodes, 0);  // out-edge iterator position (CSR index) of visited nodes
    std::vector<int64_t> path;             // find_cycle's `edges`: the active path, as CSR indices
    std::vector<int64_t> ckpt;             // per path edge: undo-log size just before it was yielded
    std::vector<int32_t> stack;            // edge_dfs stack: the start node, then the path heads
    std::vector<int32_t> seen_list;
    std::vector<Event> log;
    std::vector<int32_t> tail_of;          // path edge -> its tail (the node whose iterator yielded it)
    int64_t nrem = 0;

    for (int32_t s = 0; s < n_nodes; ++s) {
        if (explored[s]) continue;
        log.clear();
        path.clear();
        ckpt.clear();
        tail_of.clear();
        seen_list.clear();
        stack.assign(1, s);
        int32_t root = s;  // find_cycle's path root (the start node; a reset re-roots at the tail)
        active[s] = 1;
        seen[s] = 1;
        seen_list.push_back(s);
        int32_t prev_head = -1;
        bool done = false;
        while (!done) {
            if (stack.empty()) {
                // no cycle reachable from s: everything seen is explored for the later starts
                for (int32_t v : seen_list) explored[v] = 1;
                active[root] = 0;
                done = true;
                break;
            }
            const int32_t cur = stack.back();
            if (!visited[cur]) {
                visited[cur] = 1;
                pos[cur] = off[cur];
                log.push_back({0, cur, 0});
            }
            int64_t q = pos[cur];
            while (q < off[cur + 1] && !alive[q]) ++q;
            if (q == off[cur + 1]) {  // iterator exhausted: pop
                if (pos[cur] != q) {
                    log.push_back({1, cur, pos[cur]});
                    pos[cur] = q;
                }
                stack.pop_back();
                continue;
            }
            // yield edge q = (cur, h)
            const int64_t mark = (int64_t)log.size();
            log.push_back({1, cur, pos[cur]});
            pos[cur] = q + 1;
            const int32_t h = head[q];
            if (explored[h]) continue;  // pushed and fully walked by edge_dfs, skipped by find_cycle
            stack.push_back(h);
            if (prev_head >= 0 && cur != prev_head) {
                // backtracking: pop the path back to the edge whose head is cur (or empty it)
                while (true) {
                    if (path.empty()) {  // popped everything: active_nodes = {tail}
                        active[root] = 0;
                        root = cur;
                        active[root] = 1;
                        break;
                    }
                    const int64_t pe = path.back();
                    path.pop_back();
                    ckpt.pop_back();
                    tail_of.pop_back();
                    active[head[pe]] = 0;
                    if (!path.empty() && head[path.back()] == cur) break;
                }
            }
            path.push_back(q);
            ckpt.push_back(mark);
            tail_of.push_back(cur);
            if (active[h]) {
                // cycle: the path suffix from the first edge leaving h; remove its weakest edge
                size_t i0 = 0;
                while (i0 < path.size() && tail_of[i0] != h) ++i0;
                size_t kmin = i0;
                for (size_t k = i0 + 1; k < path.size(); ++k)
                    if (weight[path[k]] < weight[path[kmin]]) kmin = k;
                const int64_t dead = path[kmin];
                const int32_t tail_of_dead = tail_of[kmin];
                removed[nrem++] = dead;
                alive[dead] = 0;
                // rewind the DFS to the moment `dead` was about to be yielded
                const int64_t target = ckpt[kmin];
                while ((int64_t)log.size() > target) {
                    const Event ev = log.back();
                    log.pop_back();
                    if (ev.kind == 0) {
                        visited[ev.node] = 0;
                    } else if (ev.kind == 1) {
                        pos[ev.node] = ev.old;
                    } else {
                        seen[ev.node] = 0;
                        seen_list.pop_back();
                    }
                }
                // heads leaving the path (not the closing edge's: that node is on the surviving path)
                for (size_t k = kmin; k + 1 < path.size(); ++k) active[head[path[k]]] = 0;
                active[root] = 1;  // (the root is unchanged since path[kmin] was yielded)
                path.resize(kmin);
                ckpt.resize(kmin);
                tail_of.resize(kmin);
                // the edge_dfs stack at that moment: the root (= the start node: only it can be on the
                // stack without being a path head) and the surviving path heads
                stack.resize(kmin + 1);
                if (kmin == 0) {
                    // the path root was the yielding node itself: active_nodes = {tail}
                    active[root] = 0;
                    root = tail_of_dead;
                    active[root] = 1;
                }
                prev_head = kmin > 0 ? head[path[kmin - 1]] : -1;
                continue;
            }
            if (!seen[h]) {
                seen[h] = 1;
                seen_list.push_back(h);
                log.push_back({2, h, 0});
            }
            active[h] = 1;
            prev_head = h;
        }
    }
    *n_removed = nrem;
    return OVL_OK;
}
