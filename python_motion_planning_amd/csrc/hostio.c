/* Host-side marshalling either side of the kernels, as a CPython extension
 * module (python_motion_planning_amd._hostio):
 *
 *  - the reference keeps a Grid's obstacles as a Python set of (x, y) tuples (utils/environment/
 *    env.py:78-80) and every plan() walks it; set_to_words / set_to_words3d turn the set into the
 *    kernels' bit-packed x-major occupancy (bit c of word c >> 5, c = x*H + y or (x*Y + y)*Z + z)
 *    in one C pass over the set (cells outside the grid are not obstacles of any grid cell);
 *  - AStar.plan returns list(CLOSED.values()) (a_star.py:64): expand_nodes rebuilds those Node
 *    objects from the kernel's closure-ordered (cell | parent_dir << 28) records, with g
 *    accumulated by Python's own `+` on the motion costs (node.py:39-41: int while every step is
 *    straight, float after the first diagonal) and h = GraphSearcher.h (graph_search.py:41-44).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

static int get_index(PyObject* o, long long* v)
{
    if (PyLong_CheckExact(o)) {
        *v = PyLong_AsLongLong(o);
        return (*v == -1 && PyErr_Occurred()) ? -1 : 0;
    }
    PyObject* i = PyNumber_Index(o); /* numpy integers */
    if (!i) return -1;
    *v = PyLong_AsLongLong(i);
    Py_DECREF(i);
    return (*v == -1 && PyErr_Occurred()) ? -1 : 0;
}

/* set_to_words(obstacles, dims (tuple of 2 or 3 ints), out: writable uint32 buffer) -> number of
 * in-grid obstacle cells set */
static PyObject* set_to_words(PyObject* self, PyObject* args)
{
    PyObject *obs, *dims_o, *out;
    if (!PyArg_ParseTuple(args, "OOO", &obs, &dims_o, &out)) return NULL;
    PyObject* dims_t = PySequence_Tuple(dims_o);
    if (!dims_t) return NULL;
    const Py_ssize_t nd = PyTuple_GET_SIZE(dims_t);
    long long dims[3] = {1, 1, 1};
    if (nd != 2 && nd != 3) {
        Py_DECREF(dims_t);
        PyErr_SetString(PyExc_ValueError, "dims must have 2 or 3 entries");
        return NULL;
    }
    for (Py_ssize_t k = 0; k < nd; k++)
        if (get_index(PyTuple_GET_ITEM(dims_t, k), &dims[k])) {
            Py_DECREF(dims_t);
            return NULL;
        }
    Py_DECREF(dims_t);
    Py_buffer buf;
    if (PyObject_GetBuffer(out, &buf, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) < 0) return NULL;
    const unsigned long long ncell = (unsigned long long)dims[0] * dims[1] * dims[2];
    if ((unsigned long long)buf.len < ((ncell + 31) / 32) * 4) {
        PyBuffer_Release(&buf);
        PyErr_SetString(PyExc_ValueError, "output buffer too small for the grid");
        return NULL;
    }
    uint32_t* w = (uint32_t*)buf.buf;
    memset(w, 0, (size_t)buf.len);
    long long count = 0;
    PyObject* it = PyObject_GetIter(obs);
    if (!it) {
        PyBuffer_Release(&buf);
        return NULL;
    }
    PyObject* item;
    while ((item = PyIter_Next(it))) {
        long long c[3] = {0, 0, 0};
        int bad = 0;
        if (PyTuple_Check(item) && PyTuple_GET_SIZE(item) == nd) {
            for (Py_ssize_t k = 0; k < nd && !bad; k++) bad = get_index(PyTuple_GET_ITEM(item, k), &c[k]);
        } else {
            PyObject* t = PySequence_Tuple(item);
            if (!t || PyTuple_GET_SIZE(t) != nd) {
                Py_XDECREF(t);
                if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "obstacle entries must have the grid's rank");
                bad = 1;
            } else {
                for (Py_ssize_t k = 0; k < nd && !bad; k++) bad = get_index(PyTuple_GET_ITEM(t, k), &c[k]);
                Py_DECREF(t);
            }
        }
        Py_DECREF(item);
        if (bad) {
            Py_DECREF(it);
            PyBuffer_Release(&buf);
            return NULL;
        }
        int in = 1;
        for (int k = 0; k < 3; k++) in &= c[k] >= 0 && c[k] < dims[k];
        if (!in) continue;
        const unsigned long long cell = ((unsigned long long)c[0] * dims[1] + c[1]) * dims[2] + c[2];
        const uint32_t bit = 1u << (cell & 31);
        if (!(w[cell >> 5] & bit)) count++;
        w[cell >> 5] |= bit;
    }
    Py_DECREF(it);
    PyBuffer_Release(&buf);
    if (PyErr_Occurred()) return NULL;
    return PyLong_FromLongLong(count);
}

/* open-addressing map cell -> (g, current tuple) of a CLOSED node (new references) */
typedef struct {
    uint32_t* key;
    PyObject** val;  /* g */
    PyObject** cur;  /* the node's current tuple: the parent tuple of the nodes it closes */
    size_t mask;
} gmap_t;

static Py_ssize_t gmap_find(const gmap_t* m, uint32_t k)
{
    size_t i = ((size_t)k * 0x9E3779B1u) & m->mask;
    while (m->val[i]) {
        if (m->key[i] == k) return (Py_ssize_t)i;
        i = (i + 1) & m->mask;
    }
    return -1;
}

static void gmap_put(gmap_t* m, uint32_t k, PyObject* g, PyObject* cur) /* new references taken */
{
    size_t i = ((size_t)k * 0x9E3779B1u) & m->mask;
    while (m->val[i]) {
        if (m->key[i] == k) {
            Py_DECREF(m->val[i]);
            Py_DECREF(m->cur[i]);
            m->val[i] = g;
            m->cur[i] = cur;
            return;
        }
        i = (i + 1) & m->mask;
    }
    m->key[i] = k;
    m->val[i] = g;
    m->cur[i] = cur;
}

static PyObject* pair(long long a, long long b)
{
    PyObject* t = PyTuple_New(2);
    if (!t) return NULL;
    PyObject* x = PyLong_FromLongLong(a);
    PyObject* y = x ? PyLong_FromLongLong(b) : NULL;
    if (!y) {
        Py_XDECREF(x);
        Py_DECREF(t);
        return NULL;
    }
    PyTuple_SET_ITEM(t, 0, x);
    PyTuple_SET_ITEM(t, 1, y);
    return t;
}

/* Byte offsets of the __slots__ members current, parent, g, h of node_cls (object members of its
 * instance layout), or 0 when the class does not keep them as plain slots: then every node is built by
 * calling the class. */
static int slot_offsets(PyObject* cls, Py_ssize_t off[4])
{
    static const char* names[4] = {"current", "parent", "g", "h"};
    if (!PyType_Check(cls)) return 0;
    for (int k = 0; k < 4; k++) {
        PyObject* d = PyObject_GetAttrString(cls, names[k]);
        if (!d) {
            PyErr_Clear();
            return 0;
        }
        const int ok = Py_IS_TYPE(d, &PyMemberDescr_Type) &&
                       ((PyMemberDescrObject*)d)->d_member->type == T_OBJECT_EX;
        off[k] = ok ? ((PyMemberDescrObject*)d)->d_member->offset : 0;
        Py_DECREF(d);
        if (!ok) return 0;
    }
    return 1;
}

/* expand_nodes(records uint32 buffer, n, H, motions_xy (8 (dx, dy) tuples), motion_g (8 objects),
 *              goal (gx, gy), kind, node_cls) -> list of node_cls(current, parent, g, h)
 * kind: 0 AStar euclidean, 1 AStar manhattan, 2 Dijkstra (h = 0), 3 GBFS euclidean (g = 0),
 *       4 GBFS manhattan.  Record: cell | dir << 28, dir 8 = the start (parent = itself, g = h = 0).
 * The drop-in Node keeps its fields in __slots__, so the objects are allocated and filled directly
 * (the attributes node_cls.__init__ would set, without running it per node); a node's parent tuple is
 * the CLOSED parent's own current tuple (equal, as the reference's). */
static PyObject* expand_nodes(PyObject* self, PyObject* args)
{
    PyObject *rec_o, *mxy, *mg_o, *goal_o, *cls;
    Py_ssize_t n;
    int H, kind;
    if (!PyArg_ParseTuple(args, "OniOOOiO", &rec_o, &n, &H, &mxy, &mg_o, &goal_o, &kind, &cls)) return NULL;
    Py_buffer buf;
    if (PyObject_GetBuffer(rec_o, &buf, PyBUF_C_CONTIGUOUS) < 0) return NULL;
    if ((Py_ssize_t)(buf.len / 4) < n || H < 1) {
        PyBuffer_Release(&buf);
        PyErr_SetString(PyExc_ValueError, "bad record buffer / H");
        return NULL;
    }
    const uint32_t* rec = (const uint32_t*)buf.buf;
    long long mx[8], my[8], gx, gy;
    PyObject* mg[8];
    for (int d = 0; d < 8; d++) {
        PyObject* t = PySequence_GetItem(mxy, d);
        if (!t) { PyBuffer_Release(&buf); return NULL; }
        PyObject* a = PySequence_GetItem(t, 0);
        PyObject* b = PySequence_GetItem(t, 1);
        Py_DECREF(t);
        int bad = !a || !b || get_index(a, &mx[d]) || get_index(b, &my[d]);
        Py_XDECREF(a);
        Py_XDECREF(b);
        mg[d] = PySequence_GetItem(mg_o, d);
        if (bad || !mg[d]) {
            for (int e = 0; e <= d; e++) Py_XDECREF(mg[e]);
            PyBuffer_Release(&buf);
            return NULL;
        }
    }
    {
        PyObject* a = PySequence_GetItem(goal_o, 0);
        PyObject* b = PySequence_GetItem(goal_o, 1);
        int bad = !a || !b || get_index(a, &gx) || get_index(b, &gy);
        Py_XDECREF(a);
        Py_XDECREF(b);
        if (bad) {
            for (int d = 0; d < 8; d++) Py_DECREF(mg[d]);
            PyBuffer_Release(&buf);
            return NULL;
        }
    }
    Py_ssize_t off[4];
    const int direct = slot_offsets(cls, off);
    PyTypeObject* tp = (PyTypeObject*)cls;
    size_t cap = 16;
    while (cap < 2 * (size_t)n + 2) cap <<= 1;
    gmap_t gm;
    gm.key = (uint32_t*)PyMem_Calloc(cap, sizeof(uint32_t));
    gm.val = (PyObject**)PyMem_Calloc(cap, sizeof(PyObject*));
    gm.cur = (PyObject**)PyMem_Calloc(cap, sizeof(PyObject*));
    gm.mask = cap - 1;
    PyObject* zero = PyLong_FromLong(0);
    PyObject* list = PyList_New(n);
    int ok = gm.key && gm.val && gm.cur && zero && list;
    /* tens of thousands of new container objects: no cyclic-GC passes while they are made */
    const int gc_was = PyGC_Disable();
    for (Py_ssize_t i = 0; ok && i < n; i++) {
        const uint32_t e = rec[i], cell = e & 0x0FFFFFFFu, d = e >> 28;
        const long long x = cell / (uint32_t)H, y = cell % (uint32_t)H;
        PyObject* cur = pair(x, y);
        PyObject *par = NULL, *g = NULL, *h = NULL;
        if (!cur) { ok = 0; break; }
        if (d == 8) {
            par = cur;
            Py_INCREF(par);
            g = zero;
            Py_INCREF(g);
            h = zero;
            Py_INCREF(h);
        } else if (d < 8) {
            const long long px = x - mx[d], py = y - my[d];
            const Py_ssize_t pi = gmap_find(&gm, (uint32_t)(px * H + py));
            if (pi >= 0) {
                par = gm.cur[pi];
                Py_INCREF(par);
            } else {
                par = pair(px, py);
            }
            if (kind == 3 || kind == 4) {  /* gbfs.py:75: node_n.g = 0 */
                g = zero;
                Py_INCREF(g);
            } else if (pi >= 0) {
                /* Python's `+` (node.py:39-41), with the int / float cases done here */
                PyObject *ga = gm.val[pi], *gb = mg[d];
                if (PyFloat_CheckExact(ga) && (PyFloat_CheckExact(gb) || PyLong_CheckExact(gb)))
                    g = PyFloat_FromDouble(PyFloat_AS_DOUBLE(ga) +
                                           (PyFloat_CheckExact(gb) ? PyFloat_AS_DOUBLE(gb) : PyLong_AsDouble(gb)));
                else
                    g = PyNumber_Add(ga, gb);
            } else {
                if (!PyErr_Occurred()) PyErr_SetString(PyExc_RuntimeError, "expand record before its parent");
            }
            if (kind == 2) {  /* dijkstra.py:74: node_n.h = 0 */
                h = zero;
                Py_INCREF(h);
            } else if (kind == 1 || kind == 4) {
                h = PyLong_FromLongLong(llabs(gx - x) + llabs(gy - y));
            } else {  /* math.hypot of integer deltas == sqrt of the exact square sum (|d| <= 16384) */
                const double dx = (double)(gx - x), dy = (double)(gy - y);
                h = PyFloat_FromDouble(sqrt(dx * dx + dy * dy));
            }
        } else {
            PyErr_SetString(PyExc_ValueError, "bad expand record");
        }
        PyObject* node = NULL;
        if (par && g && h) {
            if (direct) {
                node = tp->tp_alloc(tp, 0);
                if (node) {
                    PyObject* v[4] = {cur, par, g, h};
                    for (int k = 0; k < 4; k++) {
                        Py_INCREF(v[k]);
                        *(PyObject**)((char*)node + off[k]) = v[k];
                    }
                }
            } else {
                node = PyObject_CallFunctionObjArgs(cls, cur, par, g, h, NULL);
            }
        }
        if (node) {
            Py_INCREF(g);
            Py_INCREF(cur);
            gmap_put(&gm, cell, g, cur);
            PyList_SET_ITEM(list, i, node);
        } else {
            ok = 0;
        }
        Py_XDECREF(cur);
        Py_XDECREF(par);
        Py_XDECREF(g);
        Py_XDECREF(h);
    }
    if (gc_was) PyGC_Enable();
    if (gm.val)
        for (size_t i = 0; i < cap; i++) {
            Py_XDECREF(gm.val[i]);
            if (gm.cur) Py_XDECREF(gm.cur[i]);
        }
    PyMem_Free(gm.key);
    PyMem_Free(gm.val);
    PyMem_Free(gm.cur);
    Py_XDECREF(zero);
    for (int d = 0; d < 8; d++) Py_DECREF(mg[d]);
    PyBuffer_Release(&buf);
    if (!ok) {
        Py_XDECREF(list);
        if (!PyErr_Occurred()) PyErr_NoMemory();
        return NULL;
    }
    return list;
}

static PyMethodDef methods[] = {
    {"set_to_words", set_to_words, METH_VARARGS,
     "set_to_words(obstacles, dims, out_uint32) -> count: bit-pack an obstacle set (x-major)"},
    {"expand_nodes", expand_nodes, METH_VARARGS,
     "expand_nodes(records, n, H, motions_xy, motion_g, goal, kind, node_cls) -> list of nodes"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_hostio", NULL, -1, methods};

PyMODINIT_FUNC PyInit__hostio(void) { return PyModule_Create(&moddef); }
