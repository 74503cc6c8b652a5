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
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>

static int take(PyObject* obj, Py_buffer* view, Py_ssize_t itemsize, const char* what) {
    if (PyObject_GetBuffer(obj, view, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0) return -1;
    if (view->itemsize != itemsize || view->len % itemsize != 0) {
        PyErr_Format(PyExc_TypeError, "%s: expected a contiguous array of %zd-byte integers", what, itemsize);
        PyBuffer_Release(view);
        return -1;
    }
    return 0;
}

static PyObject* build(PyObject* self, PyObject* args) {
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

static PyMethodDef methods[] = {
    {"build", build, METH_VARARGS, "build(names, u, v, weight, end) -> (node, succ, pred) dicts of a networkx DiGraph"},
    {"csr", csr, METH_VARARGS, "csr(nodes, adj[, more int types]) -> (off int64, heads int32, weights int64) bytearrays"},
    {"remove_edges", remove_edges, METH_VARARGS, "remove_edges(succ, pred, nodes, tails, heads): bulk remove_edge"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_digraph", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__digraph(void) { return PyModule_Create(&module); }
