/*
 * ovl_digraph.c — the networkx DiGraph adjacency of the overlap graph, built in C (CPython extension
 * ovlgraph._digraph; host code, SURVEY.md §8f rank 2: edge materialisation).
 *
 * construct_overlap_graph_nx_k (overlapGraphs.py:55-60) adds one edge per (pair, copy of a, copy of b)
 * with networkx's add_edge: ~3 µs per edge in Python.  ovlgraph.overlapGraphs.assemble_graph_direct
 * expands the scored pairs into edge arrays (u, v node ids in insertion order, weight, end_position) and
 * this module builds exactly the dicts add_edge would have built:
 *   node[name] = {}                                   for every node in node order (overlapGraphs.py:25-28)
 *   d = {"weight": w, "end_position": e}              one attribute dict per edge,
 *   succ[names[u]][names[v]] = d; pred[names[v]][names[u]] = d   shared by both views, edges in global order
 * so successor, predecessor and edge-data views read identically to networkx's own construction.
 *
 *   build(names: list[str], u: int64[n], v: int64[n], weight: int32[n], end: int32[n][, shared: dict])
 *       -> (node, succ, pred)
 *
 * and, for remove_cycles_from_graph (overlapGraphs.py:106-130; the replay itself is ovl_remove_cycles in
 * ovl_graph.cpp), the two per-edge passes around the replay:
 *   csr(nodes, adj) -> (off, heads, weights)          the successor lists as CSR, in DFS visiting order
 *   remove_edges(succ, pred, nodes, tails, heads)      the replay's removals, in order, as remove_edge does
 *
 * Straight from the scored pair columns (ovlgraph.overlapGraphs.OverlapEdges; the lazy DiGraph), with no edge
 * arrays in between:
 *   overlap_csr(counts, a, b, score[, keep]) -> (off, heads, weights)
 *       the graph's successor lists as CSR: node first[r] + c is copy c of read r (overlapGraphs.py:25-28);
 *       its row is, for each kept pair p with a[p] == r in list order, the copies of b[p] (:55-60)
 *   build_overlap(names, counts, a, b, score, end[, keep[, alive[, shared]]]) -> (node, succ, pred)
 *       the dicts build() makes from the expanded edges, for the edges whose CSR index is alive only (the
 *       survivors of the cycle removal, in the reference's insertion order)
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <string.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

static int take(PyObject* obj, Py_buffer* view, Py_ssize_t itemsize, const char* what) {
    if (PyObject_GetBuffer(obj, view, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0) return -1;
    if (view->itemsize != itemsize || view->len % itemsize != 0) {
        PyErr_Format(PyExc_TypeError, "%s: expected a contiguous array of %zd-byte integers", what, itemsize);
        PyBuffer_Release(view);
        return -1;
    }
    return 0;
}

/* Attribute dicts: a copy of the two-key template with its values set.  On CPython 3.10 a split-table
   template (PEP 412 key-sharing: an instance __dict__) is copied with its values array, and the two values
   are written into that array directly (indices iw / ie of the template's key table, found once by
   attr_slots) instead of two PyDict_SetItem lookups; any other dict takes the SetItem path. */
static void attr_slots(PyObject* tmpl, PyObject* kw, PyObject* ke, Py_ssize_t* iw, Py_ssize_t* ie) {
    *iw = *ie = -1;
#if PY_VERSION_HEX >= 0x030A0000 && PY_VERSION_HEX < 0x030B0000
    if (((PyDictObject*)tmpl)->ma_values == NULL || PyDict_GET_SIZE(tmpl) != 2) return;
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    while (PyDict_Next(tmpl, &pos, &k, &v)) {  /* (split table: pos - 1 is the slot in ma_values) */
        if (k == kw) *iw = pos - 1;
        else if (k == ke) *ie = pos - 1;
    }
    if (*iw < 0 || *ie < 0) *iw = *ie = -1;
#else
    (void)tmpl; (void)kw; (void)ke;
#endif
}

static PyObject* new_attr(PyObject* tmpl, PyObject* kw, PyObject* ke, Py_ssize_t iw, Py_ssize_t ie, PyObject* wv,
                          PyObject* ev) {
    PyObject* d = PyDict_Copy(tmpl);
    if (!d) return NULL;
#if PY_VERSION_HEX >= 0x030A0000 && PY_VERSION_HEX < 0x030B0000
    PyObject** vals = ((PyDictObject*)d)->ma_values;
    if (iw >= 0 && vals) {
        Py_INCREF(wv);
        Py_XSETREF(vals[iw], wv);
        Py_INCREF(ev);
        Py_XSETREF(vals[ie], ev);
        return d;
    }
#endif
    if (PyDict_SetItem(d, kw, wv) || PyDict_SetItem(d, ke, ev)) {
        Py_DECREF(d);
        return NULL;
    }
    return d;
}

static PyObject* build_impl(PyObject* self, PyObject* args) {
    (void)self;
    PyObject *names, *ou, *ov, *ow, *oe, *shared = NULL;
    if (!PyArg_ParseTuple(args, "O!OOOO|O!", &PyList_Type, &names, &ou, &ov, &ow, &oe, &PyDict_Type, &shared))
        return NULL;
    Py_buffer bu, bv, bw, be;
    if (take(ou, &bu, 8, "u") != 0) return NULL;
    if (take(ov, &bv, 8, "v") != 0) { PyBuffer_Release(&bu); return NULL; }
    if (take(ow, &bw, 4, "weight") != 0) { PyBuffer_Release(&bu); PyBuffer_Release(&bv); return NULL; }
    if (take(oe, &be, 4, "end") != 0) {
        PyBuffer_Release(&bu); PyBuffer_Release(&bv); PyBuffer_Release(&bw);
        return NULL;
    }
    PyObject *node = NULL, *succ = NULL, *pred = NULL, *kw = NULL, *ke = NULL, *tmpl = NULL, *out = NULL;
    PyObject** sin = NULL;
    PyObject** pin = NULL;
    Py_ssize_t* deg = NULL;
    const Py_ssize_t n_nodes = PyList_GET_SIZE(names);
    const Py_ssize_t n = bu.len / 8;
    if (bv.len / 8 != n || bw.len / 4 != n || be.len / 4 != n) {
        PyErr_SetString(PyExc_ValueError, "u, v, weight and end must have the same length");
        goto done;
    }
    node = PyDict_New();
    succ = PyDict_New();
    pred = PyDict_New();
    kw = PyUnicode_InternFromString("weight");
    ke = PyUnicode_InternFromString("end_position");
    sin = (PyObject**)PyMem_Malloc(sizeof(PyObject*) * (size_t)(n_nodes ? n_nodes : 1));
    pin = (PyObject**)PyMem_Malloc(sizeof(PyObject*) * (size_t)(n_nodes ? n_nodes : 1));
    if (!node || !succ || !pred || !kw || !ke || !sin || !pin) { PyErr_NoMemory(); goto done; }
    const int64_t* u = (const int64_t*)bu.buf;
    const int64_t* v = (const int64_t*)bv.buf;
    const int32_t* w = (const int32_t*)bw.buf;
    const int32_t* e = (const int32_t*)be.buf;
    /* out- and in-degrees first, so every successor / predecessor dict is created at its final size
       (no rehash while it fills) */
    deg = (Py_ssize_t*)PyMem_Calloc((size_t)(2 * n_nodes + 1), sizeof(Py_ssize_t));
    if (!deg) { PyErr_NoMemory(); goto done; }
    for (Py_ssize_t k = 0; k < n; ++k) {
        if (u[k] < 0 || u[k] >= n_nodes || v[k] < 0 || v[k] >= n_nodes) {
            PyErr_Format(PyExc_IndexError, "edge %zd: node id outside [0, %zd)", k, n_nodes);
            goto done;
        }
        ++deg[u[k]];
        ++deg[n_nodes + v[k]];
    }
    for (Py_ssize_t i = 0; i < n_nodes; ++i) {
        PyObject* name = PyList_GET_ITEM(names, i);
        PyObject* a = PyDict_New();
        PyObject* s = _PyDict_NewPresized(deg[i]);
        PyObject* p = _PyDict_NewPresized(deg[n_nodes + i]);
        if (!a || !s || !p || PyDict_SetItem(node, name, a) || PyDict_SetItem(succ, name, s) ||
            PyDict_SetItem(pred, name, p)) {
            Py_XDECREF(a); Py_XDECREF(s); Py_XDECREF(p);
            goto done;
        }
        Py_DECREF(a);
        Py_DECREF(s);
        Py_DECREF(p);
        sin[i] = s;  /* borrowed: succ / pred hold the references */
        pin[i] = p;
    }
    /* attribute dicts are copies of one two-key template with the values replaced in place, cheaper than
       growing an empty dict by two inserts.  With `shared` (an instance __dict__ holding exactly the two keys,
       PEP 412 key-sharing) every copy shares the template's key table and owns only its values: 104 instead
       of 232 bytes per edge, and still an ordinary dict (a key added later converts that one dict) */
    if (shared && PyDict_GET_SIZE(shared) == 2 && PyDict_Contains(shared, kw) == 1 && PyDict_Contains(shared, ke) == 1) {
        tmpl = shared;
        Py_INCREF(tmpl);
    } else {
        tmpl = PyDict_New();
        if (!tmpl || PyDict_SetItem(tmpl, kw, Py_None) || PyDict_SetItem(tmpl, ke, Py_None)) goto done;
    }
    for (Py_ssize_t k = 0; k < n; ++k) {
        PyObject* d = PyDict_Copy(tmpl);
        PyObject* wv = PyLong_FromLong(w[k]);
        PyObject* ev = PyLong_FromLong(e[k]);
        int bad = !d || !wv || !ev || PyDict_SetItem(d, kw, wv) || PyDict_SetItem(d, ke, ev) ||
                  PyDict_SetItem(sin[u[k]], PyList_GET_ITEM(names, v[k]), d) ||
                  PyDict_SetItem(pin[v[k]], PyList_GET_ITEM(names, u[k]), d);
        Py_XDECREF(wv);
        Py_XDECREF(ev);
        Py_XDECREF(d);
        if (bad) goto done;
    }
    out = PyTuple_Pack(3, node, succ, pred);
done:
    PyMem_Free(sin);
    PyMem_Free(pin);
    PyMem_Free(deg);
    Py_XDECREF(node);
    Py_XDECREF(succ);
    Py_XDECREF(pred);
    Py_XDECREF(tmpl);
    Py_XDECREF(kw);
    Py_XDECREF(ke);
    PyBuffer_Release(&bu);
    PyBuffer_Release(&bv);
    PyBuffer_Release(&bw);
    PyBuffer_Release(&be);
    return out;
}

/* The integer value of an edge's "weight" (an int, not a bool, or an instance of `more`, e.g. numpy.integer),
 * as remove_cycles_from_graph requires; -1 with an exception set on a missing or non-integer weight. */
static int weight_of(PyObject* attrs, PyObject* kw, PyObject* more, long long* out) {
    PyObject* w = PyDict_Check(attrs) ? PyDict_GetItemWithError(attrs, kw) : NULL;
    if (!w) {
        if (!PyErr_Occurred()) PyErr_SetObject(PyExc_KeyError, kw);
        return -1;
    }
    if (PyBool_Check(w)) goto bad;
    if (PyLong_Check(w)) {
        *out = PyLong_AsLongLong(w);
        return (*out == -1 && PyErr_Occurred()) ? -1 : 0;
    }
    if (more && PyObject_IsInstance(w, more) == 1) {
        PyObject* iv = PyNumber_Index(w);
        if (!iv) goto bad;
        *out = PyLong_AsLongLong(iv);
        Py_DECREF(iv);
        return (*out == -1 && PyErr_Occurred()) ? -1 : 0;
    }
bad:
    PyErr_Clear();
    PyErr_SetString(PyExc_TypeError, "remove_cycles_from_graph needs an integer 'weight' on every edge");
    return -1;
}

/* csr(nodes, adj[, more]) -> (off, heads, weights): the graph's successor lists as CSR in node order and, per node,
 * in adjacency order (the order networkx's DFS visits them): off int64[n+1], heads int32[E] (node indices),
 * weights int64[E], as bytearrays; None when a row is not exactly a dict (the caller's Python passes then).
 * One pass in C instead of three Python generators over 10^6-10^7 edges. */
static PyObject* csr(PyObject* self, PyObject* args) {
    (void)self;
    PyObject *nodes, *adj, *more = NULL;
    if (!PyArg_ParseTuple(args, "O!O!|O", &PyList_Type, &nodes, &PyDict_Type, &adj, &more)) return NULL;
    const Py_ssize_t n_nodes = PyList_GET_SIZE(nodes);
    PyObject *index = NULL, *boff = NULL, *bheads = NULL, *bw = NULL, *kw = NULL, *out = NULL;
    PyObject** rows = (PyObject**)PyMem_Malloc(sizeof(PyObject*) * (size_t)(n_nodes ? n_nodes : 1));
    index = PyDict_New();
    kw = PyUnicode_InternFromString("weight");
    boff = PyByteArray_FromStringAndSize(NULL, (Py_ssize_t)(8 * (n_nodes + 1)));
    if (!rows || !index || !kw || !boff) { if (!PyErr_Occurred()) PyErr_NoMemory(); goto done; }
    int64_t* off = (int64_t*)PyByteArray_AS_STRING(boff);
    off[0] = 0;
    for (Py_ssize_t i = 0; i < n_nodes; ++i) {
        PyObject* name = PyList_GET_ITEM(nodes, i);
        PyObject* iv = PyLong_FromSsize_t(i);
        if (!iv || PyDict_SetItem(index, name, iv)) { Py_XDECREF(iv); goto done; }
        Py_DECREF(iv);
        PyObject* row = PyDict_GetItemWithError(adj, name);
        if (!row) { if (!PyErr_Occurred()) PyErr_SetObject(PyExc_KeyError, name); goto done; }
        if (!PyDict_CheckExact(row)) {  /* a dict subclass may iterate in another order: caller's fallback */
            out = Py_None;
            Py_INCREF(out);
            goto done;
        }
        rows[i] = row;  /* borrowed: adj holds it */
        off[i + 1] = off[i] + PyDict_GET_SIZE(row);
    }
    const int64_t n_edges = off[n_nodes];
    bheads = PyByteArray_FromStringAndSize(NULL, (Py_ssize_t)(4 * (n_edges ? n_edges : 1)));
    bw = PyByteArray_FromStringAndSize(NULL, (Py_ssize_t)(8 * (n_edges ? n_edges : 1)));
    if (!bheads || !bw) goto done;
    int32_t* heads = (int32_t*)PyByteArray_AS_STRING(bheads);
    long long* wts = (long long*)PyByteArray_AS_STRING(bw);
    int64_t e = 0;
    for (Py_ssize_t i = 0; i < n_nodes; ++i) {
        Py_ssize_t pos = 0;
        PyObject *v, *attrs;
        while (PyDict_Next(rows[i], &pos, &v, &attrs)) {
            PyObject* iv = PyDict_GetItemWithError(index, v);
            if (!iv) { if (!PyErr_Occurred()) PyErr_SetObject(PyExc_KeyError, v); goto done; }
            heads[e] = (int32_t)PyLong_AsLong(iv);
            if (weight_of(attrs, kw, more, &wts[e]) != 0) goto done;
            ++e;
        }
    }
    out = PyTuple_Pack(3, boff, bheads, bw);
done:
    PyMem_Free(rows);
    Py_XDECREF(index);
    Py_XDECREF(kw);
    Py_XDECREF(boff);
    Py_XDECREF(bheads);
    Py_XDECREF(bw);
    return out;
}

/* remove_edges(succ, pred, nodes, tails: int64[k], heads: int64[k]): for each i in order,
 * del succ[nodes[tails[i]]][nodes[heads[i]]]; del pred[nodes[heads[i]]][nodes[tails[i]]] -- networkx's
 * DiGraph.remove_edge without its per-call cache clear (the caller clears once).  KeyError if an edge is
 * absent (edges before it stay removed, as with a loop of remove_edge). */
static PyObject* remove_edges(PyObject* self, PyObject* args) {
    (void)self;
    PyObject *succ, *pred, *nodes, *ot, *oh;
    if (!PyArg_ParseTuple(args, "O!O!O!OO", &PyDict_Type, &succ, &PyDict_Type, &pred, &PyList_Type, &nodes, &ot, &oh))
        return NULL;
    Py_buffer bt, bh;
    if (take(ot, &bt, 8, "tails") != 0) return NULL;
    if (take(oh, &bh, 8, "heads") != 0) { PyBuffer_Release(&bt); return NULL; }
    PyObject* ret = NULL;
    const Py_ssize_t n_nodes = PyList_GET_SIZE(nodes);
    const Py_ssize_t k = bt.len / 8;
    const int64_t* t = (const int64_t*)bt.buf;
    const int64_t* h = (const int64_t*)bh.buf;
    if (bh.len / 8 != k) { PyErr_SetString(PyExc_ValueError, "tails and heads must have the same length"); goto done; }
    for (Py_ssize_t i = 0; i < k; ++i) {
        if (t[i] < 0 || t[i] >= n_nodes || h[i] < 0 || h[i] >= n_nodes) {
            PyErr_Format(PyExc_IndexError, "edge %zd: node index outside [0, %zd)", i, n_nodes);
            goto done;
        }
        PyObject* u = PyList_GET_ITEM(nodes, t[i]);
        PyObject* v = PyList_GET_ITEM(nodes, h[i]);
        PyObject* su = PyDict_GetItemWithError(succ, u);
        PyObject* pv = su ? PyDict_GetItemWithError(pred, v) : NULL;
        if (!su || !pv || !PyDict_Check(su) || !PyDict_Check(pv) || PyDict_DelItem(su, v) || PyDict_DelItem(pv, u)) {
            if (!PyErr_Occurred()) PyErr_Format(PyExc_KeyError, "edge %zd is not in the graph", i);
            goto done;
        }
    }
    ret = Py_None;
    Py_INCREF(ret);
done:
    PyBuffer_Release(&bt);
    PyBuffer_Release(&bh);
    return ret;
}

/* The CSR layout of the overlap graph from the pair columns.  Pairs are grouped by read a (counting sort,
 * list order kept inside a group); row u = first[r] + c of read r has len rowlen[r] = sum of counts[b[p]] over
 * the group, the same for every copy c; pair p's edges sit at off[u] + pstart[p] + cb.  Returns 0, or -1 with
 * an exception set. */
typedef struct {
    Py_ssize_t R, P, N;
    int64_t E;
    int64_t* first;   /* R + 1 */
    int64_t* goff;    /* R + 1: group offsets into plist */
    int64_t* plist;   /* kept pairs grouped by a */
    int64_t* rowlen;  /* R */
    int64_t* pstart;  /* P (kept pairs) */
    int64_t* off;     /* N + 1 */
} Layout;

static void layout_free(Layout* L) {
    PyMem_Free(L->first);
    PyMem_Free(L->goff);
    PyMem_Free(L->plist);
    PyMem_Free(L->rowlen);
    PyMem_Free(L->pstart);
    PyMem_Free(L->off);
    memset(L, 0, sizeof(*L));
}

static int layout(Layout* L, const int32_t* counts, Py_ssize_t R, const int32_t* a, const int32_t* b, Py_ssize_t P,
                  const uint8_t* keep) {
    memset(L, 0, sizeof(*L));
    L->R = R;
    L->P = P;
    L->first = (int64_t*)PyMem_Calloc((size_t)R + 1, sizeof(int64_t));
    L->goff = (int64_t*)PyMem_Calloc((size_t)R + 1, sizeof(int64_t));
    L->plist = (int64_t*)PyMem_Malloc(sizeof(int64_t) * (size_t)(P ? P : 1));
    L->rowlen = (int64_t*)PyMem_Calloc((size_t)(R ? R : 1), sizeof(int64_t));
    L->pstart = (int64_t*)PyMem_Calloc((size_t)(P ? P : 1), sizeof(int64_t));
    if (!L->first || !L->goff || !L->plist || !L->rowlen || !L->pstart) { PyErr_NoMemory(); return -1; }
    for (Py_ssize_t r = 0; r < R; ++r) {
        if (counts[r] < 0) { PyErr_SetString(PyExc_ValueError, "negative copy count"); return -1; }
        L->first[r + 1] = L->first[r] + counts[r];
    }
    L->N = (Py_ssize_t)L->first[R];
    for (Py_ssize_t p = 0; p < P; ++p) {
        if (a[p] < 0 || a[p] >= R || b[p] < 0 || b[p] >= R) {
            PyErr_Format(PyExc_IndexError, "pair %zd: read index outside [0, %zd)", p, R);
            return -1;
        }
        if (keep && !keep[p]) continue;
        ++L->goff[a[p] + 1];
    }
    for (Py_ssize_t r = 0; r < R; ++r) L->goff[r + 1] += L->goff[r];
    int64_t* fill = (int64_t*)PyMem_Malloc(sizeof(int64_t) * (size_t)(R ? R : 1));
    if (!fill) { PyErr_NoMemory(); return -1; }
    memcpy(fill, L->goff, sizeof(int64_t) * (size_t)R);
    for (Py_ssize_t p = 0; p < P; ++p) {
        if (keep && !keep[p]) continue;
        const int32_t r = a[p];
        L->plist[fill[r]++] = p;
        L->pstart[p] = L->rowlen[r];
        L->rowlen[r] += counts[b[p]];
    }
    PyMem_Free(fill);
    L->off = (int64_t*)PyMem_Malloc(sizeof(int64_t) * ((size_t)L->N + 1));
    if (!L->off) { PyErr_NoMemory(); return -1; }
    L->off[0] = 0;
    for (Py_ssize_t r = 0; r < R; ++r)
        for (int64_t u = L->first[r]; u < L->first[r + 1]; ++u) L->off[u + 1] = L->off[u] + L->rowlen[r];
    L->E = L->off[L->N];
    return 0;
}

/* the columns of overlap_csr / build_overlap: counts, a, b (int32) and the optional keep mask (uint8 or None) */
typedef struct {
    Py_buffer c, a, b, k;
    int has_k;
} Cols;

static void cols_release(Cols* C) {
    if (C->c.obj) PyBuffer_Release(&C->c);
    if (C->a.obj) PyBuffer_Release(&C->a);
    if (C->b.obj) PyBuffer_Release(&C->b);
    if (C->has_k && C->k.obj) PyBuffer_Release(&C->k);
}

static int cols_take(Cols* C, PyObject* oc, PyObject* oa, PyObject* ob, PyObject* ok) {
    memset(C, 0, sizeof(*C));
    if (take(oc, &C->c, 4, "counts") || take(oa, &C->a, 4, "a") || take(ob, &C->b, 4, "b")) return -1;
    if (C->a.len != C->b.len) { PyErr_SetString(PyExc_ValueError, "a and b must have the same length"); return -1; }
    if (ok && ok != Py_None) {
        if (take(ok, &C->k, 1, "keep")) return -1;
        C->has_k = 1;
        if (C->k.len != C->a.len / 4) { PyErr_SetString(PyExc_ValueError, "keep must have one entry per pair"); return -1; }
    }
    return 0;
}

static PyObject* overlap_csr(PyObject* self, PyObject* args) {
    (void)self;
    PyObject *oc, *oa, *ob, *os, *ok = NULL;
    if (!PyArg_ParseTuple(args, "OOOO|O", &oc, &oa, &ob, &os, &ok)) return NULL;
    Cols C;
    Py_buffer bs;
    memset(&bs, 0, sizeof(bs));
    Layout L;
    memset(&L, 0, sizeof(L));
    PyObject *boff = NULL, *bh = NULL, *bw = NULL, *out = NULL;
    if (cols_take(&C, oc, oa, ob, ok) || take(os, &bs, 4, "score")) goto done;
    if (bs.len != C.a.len) { PyErr_SetString(PyExc_ValueError, "score must have one entry per pair"); goto done; }
    {
        const int32_t* counts = (const int32_t*)C.c.buf;
        const int32_t* a = (const int32_t*)C.a.buf;
        const int32_t* b = (const int32_t*)C.b.buf;
        const int32_t* sc = (const int32_t*)bs.buf;
        if (layout(&L, counts, C.c.len / 4, a, b, C.a.len / 4, C.has_k ? (const uint8_t*)C.k.buf : NULL)) goto done;
        boff = PyByteArray_FromStringAndSize((const char*)L.off, (Py_ssize_t)(8 * ((size_t)L.N + 1)));
        bh = PyByteArray_FromStringAndSize(NULL, (Py_ssize_t)(4 * (L.E ? L.E : 1)));
        bw = PyByteArray_FromStringAndSize(NULL, (Py_ssize_t)(8 * (L.E ? L.E : 1)));
        if (!boff || !bh || !bw) goto done;
        int32_t* heads = (int32_t*)PyByteArray_AS_STRING(bh);
        int64_t* wts = (int64_t*)PyByteArray_AS_STRING(bw);
        for (Py_ssize_t r = 0; r < L.R; ++r) {
            if (L.first[r + 1] == L.first[r]) continue;
            const int64_t u0 = L.first[r];
            int64_t e = L.off[u0];
            for (int64_t g = L.goff[r]; g < L.goff[r + 1]; ++g) {
                const int64_t p = L.plist[g];
                const int64_t v0 = L.first[b[p]];
                for (int32_t cb = 0; cb < counts[b[p]]; ++cb, ++e) {
                    heads[e] = (int32_t)(v0 + cb);
                    wts[e] = sc[p];
                }
            }
            /* every other copy of read r has the same row */
            for (int64_t u = u0 + 1; u < L.first[r + 1]; ++u) {
                memcpy(heads + L.off[u], heads + L.off[u0], sizeof(int32_t) * (size_t)L.rowlen[r]);
                memcpy(wts + L.off[u], wts + L.off[u0], sizeof(int64_t) * (size_t)L.rowlen[r]);
            }
        }
        out = PyTuple_Pack(3, boff, bh, bw);
    }
done:
    layout_free(&L);
    cols_release(&C);
    if (bs.obj) PyBuffer_Release(&bs);
    Py_XDECREF(boff);
    Py_XDECREF(bh);
    Py_XDECREF(bw);
    return out;
}

/* Python ints for edge attributes: one object per distinct value in [kIntLo, kIntHi) (scores <= 10 * l and end
 * positions <= l for the reads of the benchmark configs), shared by every edge that carries it, instead of two
 * allocations per pair; values outside the range are created per pair. */
enum { kIntLo = -4096, kIntHi = 8192 };

static PyObject* int_of(PyObject** cache, long v) {
    if (v >= kIntLo && v < kIntHi) {
        PyObject** slot = &cache[v - kIntLo];
        if (!*slot) *slot = PyLong_FromLong(v);
        Py_XINCREF(*slot);
        return *slot;
    }
    return PyLong_FromLong(v);
}

static PyObject* build_overlap_impl(PyObject* self, PyObject* args) {
    (void)self;
    PyObject *names, *oc, *oa, *ob, *os, *oe, *ok = NULL, *oalive = NULL, *shared = NULL;
    if (!PyArg_ParseTuple(args, "O!OOOOO|OOO!", &PyList_Type, &names, &oc, &oa, &ob, &os, &oe, &ok, &oalive,
                          &PyDict_Type, &shared))
        return NULL;
    Cols C;
    memset(&C, 0, sizeof(C));
    Py_buffer bs, be, bal;
    memset(&bs, 0, sizeof(bs));
    memset(&be, 0, sizeof(be));
    memset(&bal, 0, sizeof(bal));
    Layout L;
    memset(&L, 0, sizeof(L));
    PyObject *node = NULL, *succ = NULL, *pred = NULL, *kw = NULL, *ke = NULL, *tmpl = NULL, *out = NULL;
    PyObject **sin = NULL, **pin = NULL;
    PyObject** ints = (PyObject**)PyMem_Calloc((size_t)(kIntHi - kIntLo), sizeof(PyObject*));
    int64_t *dout = NULL, *din = NULL;
    if (!ints) { PyErr_NoMemory(); goto done; }
    if (cols_take(&C, oc, oa, ob, ok) || take(os, &bs, 4, "score") || take(oe, &be, 4, "end")) goto done;
    if (bs.len != C.a.len || be.len != C.a.len) {
        PyErr_SetString(PyExc_ValueError, "score and end must have one entry per pair");
        goto done;
    }
    {
        const int32_t* counts = (const int32_t*)C.c.buf;
        const int32_t* a = (const int32_t*)C.a.buf;
        const int32_t* b = (const int32_t*)C.b.buf;
        const int32_t* sc = (const int32_t*)bs.buf;
        const int32_t* en = (const int32_t*)be.buf;
        const uint8_t* keep = C.has_k ? (const uint8_t*)C.k.buf : NULL;
        if (layout(&L, counts, C.c.len / 4, a, b, C.a.len / 4, keep)) goto done;
        const Py_ssize_t n_nodes = PyList_GET_SIZE(names);
        if (n_nodes != L.N) {
            PyErr_Format(PyExc_ValueError, "%zd names for %zd nodes", n_nodes, L.N);
            goto done;
        }
        const uint8_t* alive = NULL;
        if (oalive && oalive != Py_None) {
            if (take(oalive, &bal, 1, "alive")) goto done;
            if (bal.len != L.E) { PyErr_SetString(PyExc_ValueError, "alive must have one entry per edge"); goto done; }
            alive = (const uint8_t*)bal.buf;
        }
        /* live degrees: every dict is created at its final size */
        dout = (int64_t*)PyMem_Calloc((size_t)(L.N ? L.N : 1), sizeof(int64_t));
        din = (int64_t*)PyMem_Calloc((size_t)(L.N ? L.N : 1), sizeof(int64_t));
        sin = (PyObject**)PyMem_Malloc(sizeof(PyObject*) * (size_t)(L.N ? L.N : 1));
        pin = (PyObject**)PyMem_Malloc(sizeof(PyObject*) * (size_t)(L.N ? L.N : 1));
        if (!dout || !din || !sin || !pin) { PyErr_NoMemory(); goto done; }
        for (Py_ssize_t g = 0; g < (Py_ssize_t)L.goff[L.R]; ++g) {
            const int64_t p = L.plist[g];
            for (int64_t u = L.first[a[p]]; u < L.first[a[p] + 1]; ++u) {
                const int64_t e0 = L.off[u] + L.pstart[p];
                for (int32_t cb = 0; cb < counts[b[p]]; ++cb)
                    if (!alive || alive[e0 + cb]) {
                        ++dout[u];
                        ++din[L.first[b[p]] + cb];
                    }
            }
        }
        node = PyDict_New();
        succ = PyDict_New();
        pred = PyDict_New();
        kw = PyUnicode_InternFromString("weight");
        ke = PyUnicode_InternFromString("end_position");
        if (!node || !succ || !pred || !kw || !ke) goto done;
        for (Py_ssize_t i = 0; i < n_nodes; ++i) {
            PyObject* name = PyList_GET_ITEM(names, i);
            PyObject* x = PyDict_New();
            PyObject* sd = _PyDict_NewPresized(dout[i]);
            PyObject* pd = _PyDict_NewPresized(din[i]);
            if (!x || !sd || !pd || PyDict_SetItem(node, name, x) || PyDict_SetItem(succ, name, sd) ||
                PyDict_SetItem(pred, name, pd)) {
                Py_XDECREF(x); Py_XDECREF(sd); Py_XDECREF(pd);
                goto done;
            }
            Py_DECREF(x);
            Py_DECREF(sd);
            Py_DECREF(pd);
            sin[i] = sd;
            pin[i] = pd;
        }
        if (shared && PyDict_GET_SIZE(shared) == 2 && PyDict_Contains(shared, kw) == 1 && PyDict_Contains(shared, ke) == 1) {
            tmpl = shared;
            Py_INCREF(tmpl);
        } else {
            tmpl = PyDict_New();
            if (!tmpl || PyDict_SetItem(tmpl, kw, Py_None) || PyDict_SetItem(tmpl, ke, Py_None)) goto done;
        }
        Py_ssize_t iw, ie;
        attr_slots(tmpl, kw, ke, &iw, &ie);
        /* one pass over the edges in global insertion order (pair, copy of a, copy of b: overlapGraphs.py:43-60):
           each attribute dict goes into its tail's successor dict and its head's predecessor dict while it is
           still in cache.  A node's successors arrive in that order too, which is its CSR row order. */
        for (Py_ssize_t p = 0; p < L.P; ++p) {
            if (keep && !keep[p]) continue;
            PyObject *wv = NULL, *ev = NULL;
            const int64_t vb = L.first[b[p]];
            for (int64_t u = L.first[a[p]]; u < L.first[a[p] + 1]; ++u) {
                const int64_t e0 = L.off[u] + L.pstart[p];
                PyObject* un = PyList_GET_ITEM(names, u);
                for (int32_t cb = 0; cb < counts[b[p]]; ++cb) {
                    if (alive && !alive[e0 + cb]) continue;
                    if (!wv) {
                        wv = int_of(ints, sc[p]);
                        ev = int_of(ints, en[p]);
                        if (!wv || !ev) { Py_XDECREF(wv); Py_XDECREF(ev); goto done; }
                    }
                    PyObject* d = new_attr(tmpl, kw, ke, iw, ie, wv, ev);
                    const int bad = !d || PyDict_SetItem(sin[u], PyList_GET_ITEM(names, vb + cb), d) ||
                                    PyDict_SetItem(pin[vb + cb], un, d);
                    Py_XDECREF(d);
                    if (bad) { Py_XDECREF(wv); Py_XDECREF(ev); goto done; }
                }
            }
            Py_XDECREF(wv);
            Py_XDECREF(ev);
        }
        out = PyTuple_Pack(3, node, succ, pred);
    }
done:
    layout_free(&L);
    cols_release(&C);
    if (bs.obj) PyBuffer_Release(&bs);
    if (be.obj) PyBuffer_Release(&be);
    if (bal.obj) PyBuffer_Release(&bal);
    if (ints) {
        for (int i = 0; i < kIntHi - kIntLo; ++i) Py_XDECREF(ints[i]);
        PyMem_Free(ints);
    }
    PyMem_Free(dout);
    PyMem_Free(din);
    PyMem_Free(sin);
    PyMem_Free(pin);
    Py_XDECREF(node);
    Py_XDECREF(succ);
    Py_XDECREF(pred);
    Py_XDECREF(tmpl);
    Py_XDECREF(kw);
    Py_XDECREF(ke);
    return out;
}

/* Out-edges that no removal can touch: remove_cycles_from_graph removes an edge only as the weakest of a cycle it
   lies on, so a node in a strongly connected component of its own (and without a live self-loop) never loses an
   out-edge again -- removals only delete edges, so components only split.  That holds for far more nodes, and far
   sooner, than the replay's own final set (nodes that can reach no cycle, or whose start's walk is over: at the
   target point 60 % of the nodes only at the end).  The helper recomputes the components of the live graph (Tarjan,
   iterative) pass after pass while the replay runs and publishes every node newly alone in its component.  It reads
   `alive` while the replay clears entries, so a pass sees a superset of the live edges; the components of a
   supergraph contain the true ones, so a node alone in a pass's graph is alone in the true graph too.  Edges into
   published nodes are skipped in later passes (such a node is on no cycle). */
typedef struct {
    const int64_t* off;
    const int32_t* heads;
    const uint8_t* alive;
    int32_t n;
    const int* stop;       /* the replay's finished flag */
    int* gate;             /* set after the first pass (else already set) */
    int32_t* nodes;        /* published nodes [0, n_pub) (release-ordered count) */
    int64_t n_pub;
    int passes;
    int ok;
} SccJob;

static void* scc_main(void* arg) {
    SccJob* j = (SccJob*)arg;
    const int32_t N = j->n;
    int32_t* index = (int32_t*)malloc(sizeof(int32_t) * (size_t)(N ? N : 1));
    int32_t* low = (int32_t*)malloc(sizeof(int32_t) * (size_t)(N ? N : 1));
    int32_t* stk = (int32_t*)malloc(sizeof(int32_t) * (size_t)(N ? N : 1));
    int32_t* cv = (int32_t*)malloc(sizeof(int32_t) * (size_t)(N ? N : 1));  /* call stack: node */
    int64_t* cp = (int64_t*)malloc(sizeof(int64_t) * (size_t)(N ? N : 1));  /* call stack: next edge */
    uint8_t* on = (uint8_t*)malloc((size_t)(N ? N : 1));
    uint8_t* alone = (uint8_t*)calloc((size_t)(N ? N : 1), 1);
    if (!index || !low || !stk || !cv || !cp || !on || !alone) goto out;
    j->ok = 1;
    while (!__atomic_load_n(j->stop, __ATOMIC_ACQUIRE)) {
        for (int32_t v = 0; v < N; ++v) index[v] = -1;
        memset(on, 0, (size_t)N);
        int32_t idx = 0, sp = 0;
        int64_t pub = j->n_pub;
        const int64_t pub0 = pub;
        for (int32_t r = 0; r < N && !__atomic_load_n(j->stop, __ATOMIC_RELAXED); ++r) {
            if (index[r] >= 0 || alone[r]) continue;
            int32_t depth = 0;
            cv[0] = r;
            cp[0] = j->off[r];
            index[r] = low[r] = idx++;
            stk[sp++] = r;
            on[r] = 1;
            while (depth >= 0) {
                const int32_t v = cv[depth];
                const int64_t end = j->off[v + 1];
                int64_t e = cp[depth];
                int descended = 0;
                for (; e < end; ++e) {
                    if (!__atomic_load_n(&j->alive[e], __ATOMIC_ACQUIRE)) continue;
                    const int32_t w = j->heads[e];
                    if (alone[w]) continue;
                    if (index[w] < 0) {
                        cp[depth] = e + 1;
                        ++depth;
                        cv[depth] = w;
                        cp[depth] = j->off[w];
                        index[w] = low[w] = idx++;
                        stk[sp++] = w;
                        on[w] = 1;
                        descended = 1;
                        break;
                    }
                    if (on[w] && index[w] < low[v]) low[v] = index[w];
                }
                if (descended) continue;
                /* v is done: the root of a component? */
                if (low[v] == index[v]) {
                    if (stk[sp - 1] == v) {
                        /* a component of one: alone unless a live self-loop */
                        int loop = 0;
                        for (int64_t f = j->off[v]; f < end && !loop; ++f)
                            loop = j->heads[f] == v && __atomic_load_n(&j->alive[f], __ATOMIC_ACQUIRE);
                        if (!loop) {
                            alone[v] = 1;
                            j->nodes[pub++] = v;
                            __atomic_store_n(&j->n_pub, pub, __ATOMIC_RELEASE);
                        }
                    }
                    int32_t x;
                    do {
                        x = stk[--sp];
                        on[x] = 0;
                    } while (x != v);
                }
                --depth;
                if (depth >= 0 && low[v] < low[cv[depth]]) low[cv[depth]] = low[v];
            }
        }
        ++j->passes;
        __atomic_store_n(j->gate, 1, __ATOMIC_RELEASE);
        if (j->n_pub == pub0) {  /* nothing new: let the replay remove more before the next pass */
            struct timespec ts = {0, 300000};
            nanosleep(&ts, NULL);
        }
    }
out:
    __atomic_store_n(j->gate, 1, __ATOMIC_RELEASE);
    free(index);
    free(low);
    free(stk);
    free(cv);
    free(cp);
    free(on);
    free(alone);
    return NULL;
}

/* A node's predecessor dict, built as a prefix of its in-edges in insertion order (kept pairs with b == its read in
   list order, then the copies of a): the cursor (pg, pt: pair group and tail copy) advances while the next in-edge's
   fate is known (its tail's successor row has passed it: dec), inserting the live ones. */
typedef struct {
    const Layout* L;
    const int32_t* a;
    const int64_t* blist;
    const int64_t* bgoff;
    const int64_t* rread;
    const int64_t* indeg;   /* in-edges of the node, live or not (the dict's presize) */
    const uint8_t* dec;     /* per edge: its fate is known (its tail's row has passed it) */
    PyObject* const* dptr;
    PyObject* names;
    PyObject** pin;
    int64_t* pg;            /* -1: complete */
    int64_t* pt;
    int64_t n_pred;
} PredCtx;

static int pred_advance(PredCtx* X, int64_t v) {
    int64_t g = X->pg[v];
    if (g < 0) return 0;
    const Py_ssize_t rv = (Py_ssize_t)X->rread[v];
    const int64_t gend = X->bgoff[rv + 1];
    const int64_t cv = v - X->L->first[rv];
    int64_t t = X->pt[v];
    while (g < gend) {
        const int64_t q = X->blist[g];
        const int64_t tend = X->L->first[X->a[q] + 1];
        for (; t < tend; ++t) {
            const int64_t e = X->L->off[t] + X->L->pstart[q] + cv;
            if (!X->dec[e]) {
                X->pg[v] = g;
                X->pt[v] = t;
                return 0;
            }
            PyObject* d = X->dptr[e];
            if (d) {
                if (!X->pin[v] && !(X->pin[v] = _PyDict_NewPresized(X->indeg[v]))) return -1;
                if (PyDict_SetItem(X->pin[v], PyList_GET_ITEM(X->names, t), d)) return -1;
            }
        }
        if (++g < gend) t = X->L->first[X->a[X->blist[g]]];
    }
    if (!X->pin[v] && !(X->pin[v] = PyDict_New())) return -1;
    X->pg[v] = -1;
    ++X->n_pred;
    return 0;
}

/* A node's successor dict, built the same way as a prefix of its out-edges in row order (kept pairs with a == its
   read in list order, then the copies of b): an out-edge's fate is known once it is removed (alive 0: removals are
   final), once its head is on no cycle (published by the replay or the component helper: no cycle can hold the
   edge, so it is never removed), or once the tail itself is published (all its out-edges final).  Each edge passed
   is marked decided and lets its head's predecessor dict advance. */
typedef struct {
    PredCtx* P;
    const int32_t* counts;
    const int32_t* b;
    const int32_t* sc;
    const int32_t* en;
    const uint8_t* alive;
    const uint8_t* pub;     /* per node: published (on no cycle) */
    const int64_t* outdeg;  /* out-edges of the node, live or not (the dict's presize) */
    PyObject** rows;
    PyObject** dptr;
    uint8_t* dec;
    int64_t* rg;            /* row cursor: pair group (-1: complete) */
    int32_t* rc;            /*             copy of b */
    PyObject** ints;
    PyObject *tmpl, *kw, *ke;
    Py_ssize_t iw, ie;
    PyObject** spec;        /* per edge: its attribute dict made ahead of its row (spec_advance), or NULL */
    int own;                /* dptr holds a reference (only when some (a, b) pair is listed twice, below) */
    int64_t n_rows;         /* complete rows */
    int64_t n_dec;          /* decided edges */
    int64_t n_ins;          /* live edges inserted */
    int64_t n_spec;         /* attribute dicts made ahead */
    int64_t n_spec_used;    /* ... and inserted */
} RowCtx;

/* advance u's row; `all`: u is published (every edge decided).  1 if it moved, 0 if not, -1 on error */
static int row_advance(RowCtx* R, int64_t u, int all) {
    int64_t g = R->rg[u];
    if (g < 0) return 0;
    const Layout* L = R->P->L;
    const Py_ssize_t r = (Py_ssize_t)R->P->rread[u];
    const int64_t gend = L->goff[r + 1];
    int32_t cb = R->rc[u];
    int moved = 0;
    while (g < gend) {
        const int64_t p = L->plist[g];
        const int64_t e0 = L->off[u] + L->pstart[p];
        const int64_t vb = L->first[R->b[p]];
        const int32_t nb = R->counts[R->b[p]];
        for (; cb < nb; ++cb) {
            const int64_t e = e0 + cb;
            const int live = __atomic_load_n(&R->alive[e], __ATOMIC_ACQUIRE);
            if (live && !all && !R->pub[vb + cb]) {
                R->rg[u] = g;
                R->rc[u] = cb;
                return moved;
            }
            if (live) {
                if (!R->rows[u] && !(R->rows[u] = _PyDict_NewPresized(R->outdeg[u]))) return -1;
                PyObject* d = R->spec[e];
                if (d) {
                    R->spec[e] = NULL;
                    ++R->n_spec_used;
                } else {
                    PyObject* wv = int_of(R->ints, R->sc[p]);
                    PyObject* ev = int_of(R->ints, R->en[p]);
                    d = wv && ev ? new_attr(R->tmpl, R->kw, R->ke, R->iw, R->ie, wv, ev) : NULL;
                    Py_XDECREF(wv);
                    Py_XDECREF(ev);
                }
                const int bad = !d || PyDict_SetItem(R->rows[u], PyList_GET_ITEM(R->P->names, vb + cb), d);
                if (bad) {
                    Py_XDECREF(d);
                    return -1;
                }
                /* dptr[e] is read by the head's predecessor cursor, which may still be short of e.  The row holds
                   the dict, so dptr borrows it -- unless some (a, b) pair is listed twice (not a list
                   overlapGraphs.py:43-52 makes, but OverlapEdges accepts it): the second replaces the row's entry
                   and would free the first dict, so then dptr keeps a reference, released at the exit */
                if (!R->own) Py_DECREF(d);
                R->dptr[e] = d;
                ++R->n_ins;
            }
            R->dec[e] = 1;
            ++R->n_dec;
            moved = 1;
            if (pred_advance(R->P, vb + cb)) return -1;
        }
        ++g;
        cb = 0;
    }
    if (!R->rows[u] && !(R->rows[u] = PyDict_New())) return -1;
    R->rg[u] = -1;
    ++R->n_rows;
    return 1;
}

/* Idle work while the replay runs: the attribute dicts of the still-undecided live out-edges of the nodes from *su on,
   made ahead of their rows (row_advance takes them), up to `budget` of them.  Making an edge's dict is about half of
   what inserting it costs, and the edges whose fate the replay decides last -- the graph's last cycles -- are
   otherwise all built after it has ended; an edge removed after its dict was made only costs that dict (released at
   the end).  Each node once, in node order.  Returns the dicts made (0: every node passed), -1 on error. */
#ifndef OVL_SPEC_AHEAD
#define OVL_SPEC_AHEAD 1 /* (0: no dicts made ahead -- an A/B build, tools/stream_ab.py) */
#endif
static int64_t spec_advance(RowCtx* R, int64_t* su, int64_t n_nodes, int64_t budget) {
    if (!OVL_SPEC_AHEAD) return 0;
    const Layout* L = R->P->L;
    int64_t made = 0;
    while (*su < n_nodes && made < budget) {
        const int64_t u = (*su)++;
        int64_t g = R->rg[u];
        if (g < 0 || R->pub[u]) continue;  /* (row complete, or published: built next) */
        const Py_ssize_t r = (Py_ssize_t)R->P->rread[u];
        const int64_t gend = L->goff[r + 1];
        int32_t cb = R->rc[u];
        for (; g < gend; ++g, cb = 0) {
            const int64_t p = L->plist[g];
            const int64_t e0 = L->off[u] + L->pstart[p];
            const int32_t nb = R->counts[R->b[p]];
            for (; cb < nb; ++cb) {
                const int64_t e = e0 + cb;
                if (R->spec[e] || !__atomic_load_n(&R->alive[e], __ATOMIC_ACQUIRE)) continue;
                PyObject* wv = int_of(R->ints, R->sc[p]);
                PyObject* ev = int_of(R->ints, R->en[p]);
                PyObject* d = wv && ev ? new_attr(R->tmpl, R->kw, R->ke, R->iw, R->ie, wv, ev) : NULL;
                Py_XDECREF(wv);
                Py_XDECREF(ev);
                if (!d) return -1;
                R->spec[e] = d;
                ++made;
            }
        }
    }
    R->n_spec += made;
    return made;
}

/* Idle work once every node has had its dicts made ahead: release the made-ahead dicts of edges the replay has
   removed since, `budget` entries of the edge array per call, cycling over it, so that few are left to release after
   the replay.  Returns the dicts released. */
static int64_t spec_reap(RowCtx* R, int64_t* re, int64_t n_edges, int64_t budget) {
    int64_t freed = 0;
    for (int64_t k = 0; k < budget && n_edges > 0; ++k) {
        const int64_t e = (*re)++;
        if (*re >= n_edges) *re = 0;
        PyObject* d = R->spec[e];
        if (d && !__atomic_load_n(&R->alive[e], __ATOMIC_ACQUIRE)) {
            R->spec[e] = NULL;
            Py_DECREF(d);
            ++freed;
        }
    }
    return freed;
}

/* The dicts the result is made of, ahead of their contents: every node's successor and predecessor dict not made yet
   (presized to its out- and in-edges, live or not) and the node-ordered top-level dicts (node attributes, succ,
   pred) holding them -- the rows and predecessor dicts are then filled in place.  Idle work while the replay runs
   (otherwise the last step after it), and made before the builder's collections of the young generations, which then
   take these 150 K dicts out of the final one's way.  0, or -1 with an exception set. */
static int make_tops(PyObject* names, int64_t n, PyObject** rows, PyObject** pin, const int64_t* outdeg,
                     const int64_t* indeg, PyObject** node, PyObject** succ, PyObject** pred) {
    PyObject* nd = PyDict_New();
    PyObject* sd = PyDict_New();
    PyObject* pd = PyDict_New();
    if (!nd || !sd || !pd) goto fail;
    for (Py_ssize_t i = 0; i < (Py_ssize_t)n; ++i) {
        if (!rows[i] && !(rows[i] = _PyDict_NewPresized(outdeg[i]))) goto fail;
        if (!pin[i] && !(pin[i] = _PyDict_NewPresized(indeg[i]))) goto fail;
        PyObject* name = PyList_GET_ITEM(names, i);
        PyObject* x = PyDict_New();
        const int bad = !x || PyDict_SetItem(nd, name, x) || PyDict_SetItem(sd, name, rows[i]) ||
                        PyDict_SetItem(pd, name, pin[i]);
        Py_XDECREF(x);
        if (bad) goto fail;
    }
    *node = nd;
    *succ = sd;
    *pred = pd;
    return 0;
fail:
    Py_XDECREF(nd);
    Py_XDECREF(sd);
    Py_XDECREF(pd);
    return -1;
}

/* build_overlap_stream(names, counts, a, b, score, end, keep, shared, replay_fn, off, heads, weights)
 *     -> (node, succ, pred, removed, n_removed)
 * remove_cycles_from_graph on a graph that is still columns, with the replay and the dicts overlapped: the replay
 * (replay_fn = the address of libovl's ovl_remove_cycles_stream) runs on a second thread over the CSR (off,
 * heads, weights: OverlapEdges.csr()), and this thread builds each node's successor dict as soon as the replay
 * publishes that node's out-edges as final (they can no longer be removed), with the edges' attribute dicts, and
 * each node's predecessor dict as soon as every tail of its in-edges is final: its in-edges in global insertion
 * order (pairs with b = its read in list order, then the copies of a: overlapGraphs.py:43-60); then the
 * node-ordered top-level dicts.  The result is build_overlap's for the alive mask of the replay; removed holds
 * the replay's removed CSR indices (int64) in removal order. */
/* The collector.  The builder runs with the collector off (millions of new objects), so the first allocation after it
   is back on collects the young generation: every row and predecessor dict built, traversing their millions of
   entries (~0.12 s at the target point on the box, the caller's time).  The builder instead collects the young
   generations itself (gc.collect(1): generations 0 and 1, so the next automatic collection stays a generation-0
   one) in idle time while the replay still runs, when these shares of the edges are decided, leaving only the
   dicts built after the last one for that first collection.  At most kGcMid times: each adds one to generation 2's
   count, whose threshold (10) arms a full collection. */
static const int kGcMid = 3;
static const double kGcAt[3] = {0.30, 0.50, 0.65};

/* the streamed builder's sweeps of its open rows, at most one per this many ms (target point, this container's CPU,
   three runs each: 0 -> 1 ms, build_overlap_stream 1.69-1.79 -> 1.49-1.60 s) */
static const double kSweepMs = 1.0;

/* OVL_TRACE_STREAM=1 (diagnostics): one stderr line per build_overlap_stream with the millisecond offsets of its
   phases (s setup done, r replay finished as seen here, with the share of the nodes whose rows were built by
   then, b dicts built, t top-level dicts), the replay thread's own time and the CPUs both threads ran on */
static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}

typedef int (*replay_stream_fn)(const int64_t*, const int32_t*, const int64_t*, int32_t, int64_t*, int64_t*,
                                uint8_t*, int32_t*, int64_t*);
typedef struct {
    replay_stream_fn fn;
    const int64_t* off;
    const int32_t* heads;
    const int64_t* w;
    int32_t n;
    int64_t* removed;
    int64_t n_removed;
    uint8_t* alive;
    int32_t* final_nodes;
    int64_t n_final;
    int rc;
    int finished;
    int gate;       /* the replay starts once this is non-zero (OVL_STREAM_SCC=2: after the helper's first pass) */
    int cpu_main;   /* the calling thread's CPU when the replay started */
    int cpu_start, cpu_end;
    double ms;      /* the replay's own duration */
} ReplayJob;

static void* replay_main(void* arg) {
    ReplayJob* j = (ReplayJob*)arg;
    while (!__atomic_load_n(&j->gate, __ATOMIC_ACQUIRE)) sched_yield();
    j->cpu_start = sched_getcpu();
    const double t0 = now_ms();
    j->rc = j->fn(j->off, j->heads, j->w, j->n, j->removed, &j->n_removed, j->alive, j->final_nodes, &j->n_final);
    j->ms = now_ms() - t0;
    j->cpu_end = sched_getcpu();
    __atomic_store_n(&j->finished, 1, __ATOMIC_RELEASE);
    return NULL;
}

static PyObject* build_overlap_stream_impl(PyObject* self, PyObject* args) {
    (void)self;
    PyObject *names, *oc, *oa, *ob, *os, *oe, *ok, *shared, *ooff, *oh, *ow;
    unsigned long long fn_addr;
    if (!PyArg_ParseTuple(args, "O!OOOOOOOKOOO", &PyList_Type, &names, &oc, &oa, &ob, &os, &oe, &ok, &shared,
                          &fn_addr, &ooff, &oh, &ow))
        return NULL;
    Cols C;
    memset(&C, 0, sizeof(C));
    Py_buffer bs, be, boff, bh, bw;
    memset(&bs, 0, sizeof(bs));
    memset(&be, 0, sizeof(be));
    memset(&boff, 0, sizeof(boff));
    memset(&bh, 0, sizeof(bh));
    memset(&bw, 0, sizeof(bw));
    Layout L;
    memset(&L, 0, sizeof(L));
    ReplayJob job;
    memset(&job, 0, sizeof(job));
    pthread_t th, scc_th;
    int started = 0, scc_started = 0;
    SccJob scc;
    memset(&scc, 0, sizeof(scc));
    /* OVL_STREAM_SCC (tests, A/B): 0 rows only as the replay publishes them (no component helper); 2 the replay
       waits for the helper's first pass (every node alone in the whole graph's components goes first) */
    const char* scc_env = getenv("OVL_STREAM_SCC");
    const int scc_on = scc_env ? atoi(scc_env) : 1;
    const char* tr_env = getenv("OVL_TRACE_STREAM");
    const int trace = tr_env && atoi(tr_env) != 0;
    const double t0 = trace ? now_ms() : 0.0;
    double t_setup = 0.0, t_replay = -1.0, t_built = 0.0;
    int64_t k_at_replay = 0, dec_at_replay = 0, ins_at_replay = 0;
    PyObject *node = NULL, *succ = NULL, *pred = NULL, *kw = NULL, *ke = NULL, *tmpl = NULL, *out = NULL;
    PyObject **rows = NULL, **dptr = NULL, **pin = NULL, **spec = NULL;
    PyObject* gc_collect = NULL;
    int own_refs = 1;  /* dptr's entries are references (until the columns are known free of repeated pairs) */
    PyObject** ints = (PyObject**)PyMem_Calloc((size_t)(kIntHi - kIntLo), sizeof(PyObject*));
    int64_t* rread = NULL;
    int64_t *bgoff = NULL, *blist = NULL, *pending = NULL, *ready = NULL, *pg = NULL, *pt = NULL, *rg = NULL;
    int64_t *outdeg = NULL, *openl = NULL;
    int32_t* rc = NULL;
    uint8_t *pubd = NULL, *dec = NULL;
    if (!ints) { PyErr_NoMemory(); goto done; }
    if (cols_take(&C, oc, oa, ob, ok) || take(os, &bs, 4, "score") || take(oe, &be, 4, "end") ||
        take(ooff, &boff, 8, "off") || take(oh, &bh, 4, "heads") || take(ow, &bw, 8, "weights"))
        goto done;
    if (bs.len != C.a.len || be.len != C.a.len) {
        PyErr_SetString(PyExc_ValueError, "score and end must have one entry per pair");
        goto done;
    }
    /* the replay needs only the CSR: start it first, and lay out the columns while it runs (the CSR is checked
       against them below; on a mismatch the replay of the caller's CSR still ends, is joined and the call fails) */
    if (boff.len < 8 || bh.len / 4 != bw.len / 8 || boff.len / 8 - 1 >= ((Py_ssize_t)1 << 31)) {
        PyErr_SetString(PyExc_ValueError, "names / CSR do not match the columns' graph");
        goto done;
    }
    {
        const int64_t E = (int64_t)(bh.len / 4), N = (int64_t)(boff.len / 8 - 1);
        job.fn = (replay_stream_fn)(uintptr_t)fn_addr;
        job.off = (const int64_t*)boff.buf;
        job.heads = (const int32_t*)bh.buf;
        job.w = (const int64_t*)bw.buf;
        job.n = (int32_t)N;
        job.removed = (int64_t*)PyMem_RawMalloc(sizeof(int64_t) * (size_t)(E ? E : 1));
        job.alive = (uint8_t*)PyMem_RawMalloc((size_t)(E ? E : 1));
        job.final_nodes = (int32_t*)PyMem_RawMalloc(sizeof(int32_t) * (size_t)(N ? N : 1));
        if (!job.removed || !job.alive || !job.final_nodes) {
            PyErr_NoMemory();
            goto done;
        }
        /* all ones before either thread starts (the replay sets it too, but on its own thread, where the component
           helper could read it first) */
        memset(job.alive, 1, (size_t)E);
        job.cpu_main = sched_getcpu();
        job.gate = scc_on != 2;
        if (pthread_create(&th, NULL, replay_main, &job) != 0) {
            PyErr_SetString(PyExc_RuntimeError, "cannot start the replay thread");
            goto done;
        }
        started = 1;
        if (trace) t_setup = now_ms() - t0;
    }
    {
        const int32_t* counts = (const int32_t*)C.c.buf;
        const int32_t* a = (const int32_t*)C.a.buf;
        const int32_t* b = (const int32_t*)C.b.buf;
        const int32_t* sc = (const int32_t*)bs.buf;
        const int32_t* en = (const int32_t*)be.buf;
        const uint8_t* keep = C.has_k ? (const uint8_t*)C.k.buf : NULL;
        if (layout(&L, counts, C.c.len / 4, a, b, C.a.len / 4, keep)) goto done;
        const Py_ssize_t n_nodes = PyList_GET_SIZE(names);
        if (n_nodes != L.N || boff.len / 8 != L.N + 1 || bh.len / 4 != L.E || bw.len / 8 != L.E ||
            L.N >= ((Py_ssize_t)1 << 31)) {
            PyErr_SetString(PyExc_ValueError, "names / CSR do not match the columns' graph");
            goto done;
        }
        const int64_t E = L.E, N = L.N;
        rows = (PyObject**)PyMem_Calloc((size_t)(N ? N : 1), sizeof(PyObject*));
        pin = (PyObject**)PyMem_Calloc((size_t)(N ? N : 1), sizeof(PyObject*));
        dptr = (PyObject**)PyMem_Calloc((size_t)(E ? E : 1), sizeof(PyObject*));
        spec = (PyObject**)PyMem_Calloc((size_t)(E ? E : 1), sizeof(PyObject*));
        rread = (int64_t*)PyMem_Malloc(sizeof(int64_t) * (size_t)(N ? N : 1));
        /* in-edges in insertion order: the kept pairs grouped by b (list order within a group) */
        bgoff = (int64_t*)PyMem_Calloc((size_t)L.R + 1, sizeof(int64_t));
        blist = (int64_t*)PyMem_Malloc(sizeof(int64_t) * (size_t)(L.P ? L.P : 1));
        pending = (int64_t*)PyMem_Calloc((size_t)(N ? N : 1), sizeof(int64_t));
        if (!rows || !pin || !dptr || !spec || !rread || !bgoff || !blist || !pending) {
            PyErr_NoMemory();
            goto done;
        }
        for (Py_ssize_t r = 0; r < L.R; ++r)
            for (int64_t u = L.first[r]; u < L.first[r + 1]; ++u) rread[u] = r;
        for (Py_ssize_t p = 0; p < L.P; ++p)
            if (!keep || keep[p]) ++bgoff[b[p] + 1];
        for (Py_ssize_t r = 0; r < L.R; ++r) bgoff[r + 1] += bgoff[r];
        {
            int64_t* fill = (int64_t*)PyMem_Malloc(sizeof(int64_t) * (size_t)(L.R ? L.R : 1));
            if (!fill) { PyErr_NoMemory(); goto done; }
            memcpy(fill, bgoff, sizeof(int64_t) * (size_t)L.R);
            for (Py_ssize_t p = 0; p < L.P; ++p)
                if (!keep || keep[p]) blist[fill[b[p]]++] = p;
            PyMem_Free(fill);
        }
        /* a node's in-edges, live or not (every copy of one read has the same in-edges) */
        for (Py_ssize_t r = 0; r < L.R; ++r) {
            int64_t k = 0;
            for (int64_t g = bgoff[r]; g < bgoff[r + 1]; ++g) k += L.first[a[blist[g]] + 1] - L.first[a[blist[g]]];
            for (int64_t v = L.first[r]; v < L.first[r + 1]; ++v) pending[v] = k;
        }
        kw = PyUnicode_InternFromString("weight");
        ke = PyUnicode_InternFromString("end_position");
        if (!kw || !ke) goto done;
        if (shared && shared != Py_None && PyDict_Check(shared) && PyDict_GET_SIZE(shared) == 2 &&
            PyDict_Contains(shared, kw) == 1 && PyDict_Contains(shared, ke) == 1) {
            tmpl = shared;
            Py_INCREF(tmpl);
        } else {
            tmpl = PyDict_New();
            if (!tmpl || PyDict_SetItem(tmpl, kw, Py_None) || PyDict_SetItem(tmpl, ke, Py_None)) goto done;
        }
        Py_ssize_t iw, ie;
        attr_slots(tmpl, kw, ke, &iw, &ie);
        {
            PyObject* gcm = PyImport_ImportModule("gc");
            if (!gcm) goto done;
            gc_collect = PyObject_GetAttrString(gcm, "collect");
            Py_DECREF(gcm);
            if (!gc_collect) goto done;
        }
        if (trace) t_setup = now_ms() - t0;  /* (s: the builder's setup done, the replay running since the start) */
        /* successors of each node as its out-edges become final (row order: kept pairs with a == its read in
           list order, then the copies of b) -- published by the replay (settled or explored nodes) or by the
           component helper (scc_main), whichever comes first; predecessors of each node once every tail of its
           in-edges is */
        if (scc_on) {
            scc.off = job.off;
            scc.heads = job.heads;
            scc.alive = job.alive;
            scc.n = (int32_t)N;
            scc.stop = &job.finished;
            scc.gate = &job.gate;
            scc.nodes = (int32_t*)PyMem_RawMalloc(sizeof(int32_t) * (size_t)(N ? N : 1));
            if (!scc.nodes) { PyErr_NoMemory(); goto done; }
            if (pthread_create(&scc_th, NULL, scc_main, &scc) != 0) {
                PyErr_SetString(PyExc_RuntimeError, "cannot start the component thread");
                goto done;
            }
            scc_started = 1;
        }
        int64_t k_done = 0, k_scc = 0, n_pub = 0, n_from_scc = 0, n_sweeps = 0;
        pg = (int64_t*)PyMem_Malloc(sizeof(int64_t) * (size_t)(N ? N : 1));
        pt = (int64_t*)PyMem_Malloc(sizeof(int64_t) * (size_t)(N ? N : 1));
        rg = (int64_t*)PyMem_Malloc(sizeof(int64_t) * (size_t)(N ? N : 1));
        rc = (int32_t*)PyMem_Calloc((size_t)(N ? N : 1), sizeof(int32_t));
        outdeg = (int64_t*)PyMem_Calloc((size_t)(N ? N : 1), sizeof(int64_t));
        pubd = (uint8_t*)PyMem_Calloc((size_t)(N ? N : 1), 1);
        dec = (uint8_t*)PyMem_Calloc((size_t)(E ? E : 1), 1);
        openl = (int64_t*)PyMem_Malloc(sizeof(int64_t) * (size_t)(N ? N : 1));
        if (!pg || !pt || !rg || !rc || !outdeg || !pubd || !dec || !openl) { PyErr_NoMemory(); goto done; }
        PredCtx X = {&L, a, blist, bgoff, rread, pending, dec, dptr, names, pin, pg, pt, 0};
        for (int64_t v = 0; v < N; ++v) {
            const Py_ssize_t rv = (Py_ssize_t)rread[v];
            pg[v] = bgoff[rv];
            pt[v] = bgoff[rv] < bgoff[rv + 1] ? L.first[a[blist[bgoff[rv]]]] : 0;
            rg[v] = L.goff[rv];
            for (int64_t g = L.goff[rv]; g < L.goff[rv + 1]; ++g) outdeg[v] += counts[b[L.plist[g]]];
            openl[v] = v;
        }
        int64_t n_open = N;
        /* some read's kept pairs list the same b twice? (then dptr owns its references, RowCtx.own) */
        int dup = 0;
        {
            int32_t* stamp = (int32_t*)PyMem_Calloc((size_t)(L.R ? L.R : 1), sizeof(int32_t));
            if (!stamp) { PyErr_NoMemory(); goto done; }
            for (Py_ssize_t r = 0; r < L.R && !dup; ++r)
                for (int64_t g = L.goff[r]; g < L.goff[r + 1]; ++g) {
                    const int32_t bb = b[L.plist[g]];
                    if (stamp[bb] == (int32_t)r + 1) { dup = 1; break; }
                    stamp[bb] = (int32_t)r + 1;
                }
            PyMem_Free(stamp);
        }
        own_refs = dup;
        RowCtx R = {&X, counts, b, sc, en, job.alive, pubd, outdeg, rows, dptr, dec, rg, rc, ints, tmpl, kw, ke, iw, ie,
                    spec, dup, 0, 0, 0, 0, 0};
        int64_t spec_u = 0;     /* spec_advance's next node */
        int64_t reap_e = 0;     /* spec_reap's next edge */
        int n_gc = 0;           /* collections of the young generations run so far (kGcMid) */
        double t_tops = -1.0;
        double t_gc = 0.0;
        double t_sweep = -1e9;  /* the last sweep's start (ms) */
        for (int64_t v = 0; v < N; ++v)
            if (pred_advance(&X, v)) goto done;  /* (completes the nodes without in-edges) */
        for (;;) {
            if (trace && t_replay < 0.0 && __atomic_load_n(&job.finished, __ATOMIC_ACQUIRE)) {
                t_replay = now_ms() - t0;
                k_at_replay = R.n_rows;
                dec_at_replay = R.n_dec;
                ins_at_replay = R.n_ins;
            }
            int64_t u = -1;
            if (k_done < __atomic_load_n(&job.n_final, __ATOMIC_ACQUIRE)) {
                u = job.final_nodes[k_done++];
            } else if (scc_started && k_scc < __atomic_load_n(&scc.n_pub, __ATOMIC_ACQUIRE)) {
                u = scc.nodes[k_scc++];
                if (!pubd[u]) ++n_from_scc;
            }
            if (u >= 0) {
                if (pubd[u]) continue;  /* (published by both) */
                pubd[u] = 1;
                ++n_pub;
                if (row_advance(&R, u, 1) < 0) goto done;
                continue;
            }
            if (__atomic_load_n(&job.finished, __ATOMIC_ACQUIRE)) {
                if (__atomic_load_n(&job.n_final, __ATOMIC_ACQUIRE) > k_done) continue;
                break;
            }
            /* nothing newly published: advance the openl rows as far as their heads allow -- at most once per
               kSweepMs (a sweep calls row_advance on every open row, hundreds of millions of calls over a run when
               repeated back to back); in between, and after a sweep that moved nothing, make attribute dicts ahead */
            if (now_ms() - t_sweep < kSweepMs) {
                if (!node) {  /* first: every row and predecessor dict and the top-level dicts, once */
                    if (make_tops(names, N, rows, pin, outdeg, pending, &node, &succ, &pred)) goto done;
                    if (trace) t_tops = now_ms() - t0;
                    continue;
                }
                if (gc_collect && n_gc < kGcMid && R.n_dec >= (int64_t)(kGcAt[n_gc] * (double)E)) {
                    /* the collector's pass over the dicts built so far, now, beside the replay (see kGcMid) */
                    const double tg = now_ms();
                    PyObject* res = PyObject_CallFunction(gc_collect, "i", 1);
                    if (!res) goto done;
                    Py_DECREF(res);
                    t_gc += now_ms() - tg;
                    ++n_gc;
                    continue;
                }
                const int64_t m = spec_advance(&R, &spec_u, N, 256);
                if (m < 0) goto done;
                if (m == 0) {
                    if (OVL_SPEC_AHEAD) (void)spec_reap(&R, &reap_e, E, 16384);
                    Py_BEGIN_ALLOW_THREADS
                    sched_yield();
                    Py_END_ALLOW_THREADS
                }
                continue;
            }
            t_sweep = now_ms();
            int moved = 0;
            int64_t keep_n = 0;
            for (int64_t i = 0; i < n_open; ++i) {
                const int64_t x = openl[i];
                if (rg[x] < 0) continue;
                const int m = row_advance(&R, x, 0);
                if (m < 0) goto done;
                moved |= m;
                if (rg[x] >= 0) openl[keep_n++] = x;
                if ((i & 255) == 255 && k_done < __atomic_load_n(&job.n_final, __ATOMIC_ACQUIRE)) {
                    /* (newly published nodes first: keep the rest of the list for the next sweep) */
                    for (int64_t j = i + 1; j < n_open; ++j) openl[keep_n++] = openl[j];
                    break;
                }
            }
            n_open = keep_n;
            ++n_sweeps;
            if (!moved) {  /* nothing to insert yet: make attribute dicts ahead, else yield */
                const int64_t m = spec_advance(&R, &spec_u, N, 256);
                if (m < 0) goto done;
                if (m == 0) {
                    Py_BEGIN_ALLOW_THREADS
                    sched_yield();
                    Py_END_ALLOW_THREADS
                }
            }
        }
        const int64_t n_rows = R.n_rows;
        const int64_t n_pred = X.n_pred;
        pthread_join(th, NULL);
        started = 0;
        if (scc_started) {
            pthread_join(scc_th, NULL);
            scc_started = 0;
        }
        if (trace) t_built = now_ms() - t0;
        if (job.rc != 0 || k_done != N || n_rows != N || n_pred != N) {
            PyErr_Format(PyExc_RuntimeError, "ovl_remove_cycles_stream failed (rc %d, %lld of %lld nodes final, "
                         "%lld predecessor dicts)", job.rc, (long long)k_done, (long long)N, (long long)n_pred);
            goto done;
        }
        if (!node && make_tops(names, N, rows, pin, outdeg, pending, &node, &succ, &pred)) goto done;
        PyObject* rem = PyBytes_FromStringAndSize((const char*)job.removed, (Py_ssize_t)(8 * job.n_removed));
        if (!rem) goto done;
        out = Py_BuildValue("(OOONL)", node, succ, pred, rem, (long long)job.n_removed);
        if (trace)
            fprintf(stderr, "ovl_stream: s=%.1f r=%.1f (%.0f%% rows, %.0f%% edges, %lld inserted) b=%.1f t=%.1f sweeps=%lld scc=%d passes=%d first=%lld "
                    "replay=%.1f cpus main %d/%d replay %d/%d spec %lld used %lld gc %d in %.1f ms tops at %.1f dec %.0f%%\n", t_setup, t_replay,
                    N ? 100.0 * (double)k_at_replay / (double)N : 100.0,
                    E ? 100.0 * (double)dec_at_replay / (double)E : 100.0, (long long)ins_at_replay, t_built, now_ms() - t0, (long long)n_sweeps,
                    scc_on, scc.passes,
                    (long long)n_from_scc, job.ms, job.cpu_main, sched_getcpu(), job.cpu_start, job.cpu_end, (long long)R.n_spec, (long long)R.n_spec_used, n_gc, t_gc, t_tops, E ? 100.0 * (double)dec_at_replay / (double)E : 0.0);
    }
done:
    if (started) {  /* an error while the replay runs: let it finish (it owns no Python objects) */
        __atomic_store_n(&job.gate, 1, __ATOMIC_RELEASE);  /* (if it still waits for the helper's first pass) */
        Py_BEGIN_ALLOW_THREADS
        pthread_join(th, NULL);
        Py_END_ALLOW_THREADS
    }
    if (scc_started) {  /* (it stops once the replay has finished) */
        Py_BEGIN_ALLOW_THREADS
        pthread_join(scc_th, NULL);
        Py_END_ALLOW_THREADS
    }
    const Py_ssize_t L_N = L.N, L_E = L.E;  /* (layout_free zeroes L) */
    layout_free(&L);
    cols_release(&C);
    if (bs.obj) PyBuffer_Release(&bs);
    if (be.obj) PyBuffer_Release(&be);
    if (boff.obj) PyBuffer_Release(&boff);
    if (bh.obj) PyBuffer_Release(&bh);
    if (bw.obj) PyBuffer_Release(&bw);
    if (ints) {
        for (int i = 0; i < kIntHi - kIntLo; ++i) Py_XDECREF(ints[i]);
        PyMem_Free(ints);
    }
    if (rows) {
        for (Py_ssize_t i = 0; i < L_N; ++i) Py_XDECREF(rows[i]);
        PyMem_Free(rows);
    }
    if (pin) {
        for (Py_ssize_t i = 0; i < L_N; ++i) Py_XDECREF(pin[i]);
        PyMem_Free(pin);
    }
    const double tc0 = trace ? now_ms() : 0.0;
    if (dptr) {
        if (own_refs)
            for (Py_ssize_t e = 0; e < L_E; ++e) Py_XDECREF(dptr[e]);
        PyMem_Free(dptr);
    }
    const double tc1 = trace ? now_ms() : 0.0;
    if (spec) {  /* (the dicts made ahead for edges the replay then removed) */
        for (Py_ssize_t e = 0; e < L_E; ++e) Py_XDECREF(spec[e]);
        PyMem_Free(spec);
    }
    Py_XDECREF(gc_collect);
    if (trace) fprintf(stderr, "ovl_stream exit: references %.1f ms, dicts made ahead and unused %.1f ms\n", tc1 - tc0,
                       now_ms() - tc1);
    PyMem_Free(rread);
    PyMem_Free(bgoff);
    PyMem_Free(blist);
    PyMem_Free(pending);
    PyMem_Free(ready);
    PyMem_Free(pg);
    PyMem_Free(pt);
    PyMem_Free(rg);
    PyMem_Free(rc);
    PyMem_Free(outdeg);
    PyMem_Free(pubd);
    PyMem_Free(dec);
    PyMem_Free(openl);
    PyMem_RawFree(scc.nodes);
    PyMem_RawFree(job.removed);
    PyMem_RawFree(job.alive);
    PyMem_RawFree(job.final_nodes);
    Py_XDECREF(node);
    Py_XDECREF(succ);
    Py_XDECREF(pred);
    Py_XDECREF(tmpl);
    Py_XDECREF(kw);
    Py_XDECREF(ke);
    return out;
}

// ----------------------------------------------------------------------------- pooled object arenas
//
// The graph's dicts (an attribute dict per edge, a row and a predecessor dict per node: ~2.3 M objects at the
// target point, ~0.4 GB) come from CPython's object arenas (256 KiB each, one mmap per arena).  Fresh arenas land on
// pages the kernel must fault in and zero, 4 KiB at a time: ~2·10^5 minor faults in a process's first removal.
// While a builder call runs (build, build_overlap, build_overlap_stream: pool_scope), an arena allocator carves
// arenas from 64 MiB regions aligned to 2 MiB and advised for transparent huge pages (far fewer faults), and arenas
// freed meanwhile go on a free list for the call's own later dicts.  The previous allocator is restored when the
// call returns, so the pool touches nothing else in the process: the graph's arenas go back to the kernel by
// CPython's own munmap when the graph is freed, and of the free list at most kPoolKeep arenas stay mapped for the
// next call (the rest are unmapped).  OVL_ARENA_POOL=0: builder calls keep CPython's allocator.
#include <sys/mman.h>

#define OVL_POOL_REGION (64u << 20)
#define OVL_POOL_MAX_REGIONS 1024
#define OVL_POOL_KEEP 256  // freed arenas kept mapped across builder calls (64 MiB of 256 KiB arenas)

static PyObjectArenaAllocator g_prev_arena;
static int g_pool_enabled = -1;   // OVL_ARENA_POOL (read once): 0 off, else on
static int g_pool_depth = 0;      // builder calls in progress (the allocator is installed while > 0)
static void* g_pool_free = NULL;  // freed pool arenas, linked through their first word
static size_t g_pool_nfree = 0;
static char* g_pool_cur = NULL;
static size_t g_pool_left = 0;
static size_t g_pool_arena = 0;  // the arena size CPython asks for (the first request's)
static char* g_region_base[OVL_POOL_MAX_REGIONS];  // ascending
static int g_regions = 0;
static size_t g_pool_mapped = 0, g_pool_reused = 0, g_pool_released = 0;

static int pool_owns(const void* p) {  // (binary search over the ascending region bases)
    int lo = 0, hi = g_regions;
    while (lo < hi) {
        const int mid = (lo + hi) / 2;
        if ((const char*)p < g_region_base[mid]) hi = mid;
        else lo = mid + 1;
    }
    return lo > 0 && (const char*)p < g_region_base[lo - 1] + OVL_POOL_REGION;
}

static void* pool_arena_alloc(void* ctx, size_t size) {
    (void)ctx;
    if (!g_pool_arena) g_pool_arena = size;
    if (size != g_pool_arena || size > OVL_POOL_REGION) return g_prev_arena.alloc(g_prev_arena.ctx, size);
    if (g_pool_free) {
        void* p = g_pool_free;
        g_pool_free = *(void**)p;
        --g_pool_nfree;
        ++g_pool_reused;
        return p;
    }
    if (g_pool_left < size) {
        if (g_regions == OVL_POOL_MAX_REGIONS) return g_prev_arena.alloc(g_prev_arena.ctx, size);
        const size_t huge = (size_t)2 << 20;
        char* m = (char*)mmap(NULL, OVL_POOL_REGION + huge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (m == (char*)MAP_FAILED) return g_prev_arena.alloc(g_prev_arena.ctx, size);
        char* a = (char*)(((uintptr_t)m + huge - 1) & ~(uintptr_t)(huge - 1));
        if (a > m) munmap(m, (size_t)(a - m));                               // trim to the aligned region
        if (a + OVL_POOL_REGION < m + OVL_POOL_REGION + huge)
            munmap(a + OVL_POOL_REGION, (size_t)(m + OVL_POOL_REGION + huge - (a + OVL_POOL_REGION)));
#ifdef MADV_HUGEPAGE
        madvise(a, OVL_POOL_REGION, MADV_HUGEPAGE);
#endif
        int i = g_regions++;
        for (; i > 0 && g_region_base[i - 1] > a; --i) g_region_base[i] = g_region_base[i - 1];
        g_region_base[i] = a;
        g_pool_cur = a;
        g_pool_left = OVL_POOL_REGION;
        g_pool_mapped += OVL_POOL_REGION;
    }
    void* p = g_pool_cur;
    g_pool_cur += size;
    g_pool_left -= size;
    return p;
}

static void pool_arena_free(void* ctx, void* p, size_t size) {
    (void)ctx;
    if (p && size == g_pool_arena && pool_owns(p)) {
        *(void**)p = g_pool_free;
        g_pool_free = p;
        ++g_pool_nfree;
        return;
    }
    g_prev_arena.free(g_prev_arena.ctx, p, size);
}

// a builder call's start / end (with the GIL held): install the pool / trim its free list and restore CPython's
static void pool_begin(void) {
    if (g_pool_enabled < 0) {
        const char* e = getenv("OVL_ARENA_POOL");
        g_pool_enabled = !(e && !strcmp(e, "0"));
    }
    if (!g_pool_enabled || g_pool_depth++ > 0) return;
    PyObjectArenaAllocator mine = {NULL, pool_arena_alloc, pool_arena_free};
    PyObject_GetArenaAllocator(&g_prev_arena);
    PyObject_SetArenaAllocator(&mine);
}

static void pool_end(void) {
    if (!g_pool_enabled || g_pool_depth == 0 || --g_pool_depth > 0) return;
    void* keep = NULL;
    void** tail = &keep;
    size_t kept = 0;
    for (void* p = g_pool_free; p;) {
        void* next = *(void**)p;
        if (kept < OVL_POOL_KEEP) {
            *tail = p;
            tail = (void**)p;
            ++kept;
        } else {
            munmap(p, g_pool_arena);  // (its addresses are never handed out again: off the list, below g_pool_cur)
            ++g_pool_released;
        }
        p = next;
    }
    *tail = NULL;
    g_pool_free = keep;
    g_pool_nfree = kept;
    PyObject_SetArenaAllocator(&g_prev_arena);
}

// stats (tests): {on: installed now, enabled, arena_bytes, mapped_bytes, reused_arenas, kept_arenas, released_arenas}
static PyObject* arena_pool(PyObject* self, PyObject* args) {
    (void)self;
    (void)args;
    return Py_BuildValue("{s:i,s:i,s:n,s:n,s:n,s:n,s:n}", "on", g_pool_depth > 0 ? 1 : 0, "enabled", g_pool_enabled,
                         "arena_bytes", (Py_ssize_t)g_pool_arena, "mapped_bytes", (Py_ssize_t)g_pool_mapped,
                         "reused_arenas", (Py_ssize_t)g_pool_reused, "kept_arenas", (Py_ssize_t)g_pool_nfree,
                         "released_arenas", (Py_ssize_t)g_pool_released);
}

// the builder entry points, each inside a pool scope
static PyObject* build_impl(PyObject* self, PyObject* args);
static PyObject* build_overlap_impl(PyObject* self, PyObject* args);
static PyObject* build_overlap_stream_impl(PyObject* self, PyObject* args);
#define OVL_POOL_SCOPED(name)                                  \
    static PyObject* name(PyObject* self, PyObject* args) {    \
        pool_begin();                                          \
        PyObject* r = name##_impl(self, args);                 \
        pool_end();                                            \
        return r;                                              \
    }
OVL_POOL_SCOPED(build)
OVL_POOL_SCOPED(build_overlap)
OVL_POOL_SCOPED(build_overlap_stream)

static PyMethodDef methods[] = {
    {"arena_pool", arena_pool, METH_VARARGS,
     "arena_pool() -> stats of the pooled, huge-page-advised object arenas builder calls allocate from"},
    {"overlap_csr", overlap_csr, METH_VARARGS,
     "overlap_csr(counts, a, b, score[, keep]) -> (off int64, heads int32, weights int64) bytearrays"},
    {"build_overlap_stream", build_overlap_stream, METH_VARARGS,
     "build_overlap_stream(names, counts, a, b, score, end, keep, shared, replay_fn, off, heads, weights) -> "
     "(node, succ, pred, removed, n_removed)"},
    {"build_overlap", build_overlap, METH_VARARGS,
     "build_overlap(names, counts, a, b, score, end[, keep[, alive[, shared]]]) -> (node, succ, pred)"},
    {"build", build, METH_VARARGS, "build(names, u, v, weight, end) -> (node, succ, pred) dicts of a networkx DiGraph"},
    {"csr", csr, METH_VARARGS, "csr(nodes, adj[, more int types]) -> (off int64, heads int32, weights int64) bytearrays"},
    {"remove_edges", remove_edges, METH_VARARGS, "remove_edges(succ, pred, nodes, tails, heads): bulk remove_edge"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_digraph", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__digraph(void) { return PyModule_Create(&module); }
