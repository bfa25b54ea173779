/* The restricted pickle VM of flame_amd.ingest (PayloadDecoder.load) in C.
 *
 * flame's channel decodes every received message with cloudpickle.loads
 * (lib/python/flame/channel.py:321-325).  flame_amd.ingest replaces that, for update
 * payloads, with a restricted zero-copy decoder; this module is its opcode loop.  It runs
 * exactly the opcode set of the Python loop in ingest.py, with the same meaning:
 *
 *   - every global goes through the decoder's allowlist (find(module, name)), every call
 *     (REDUCE, NEWOBJ) through its checked call(fn, args) -- nothing outside the allowlist
 *     is resolved or executed, BUILD with a state is refused, persistent ids only inside a
 *     storage stream (persistent_load);
 *   - BINBYTES / SHORT_BINBYTES / BINBYTES8 as the argument of torch.storage._load_from_bytes
 *     (span_marker on top of the stack) push a span (span_cls(start, n)) of the buffer, never
 *     a copy -- tensor bytes stay where they are in the payload; any other bytes value is a
 *     bytes object.
 *
 * Every read is bounds-checked against the buffer; a payload that runs past its end, pops
 * an empty stack or mark list, or references a missing memo entry raises
 * pickle.UnpicklingError("malformed update payload: ...").  Python-level exceptions raised
 * by find / call / persistent_load propagate unchanged, as in the Python loop.
 *
 *     load(buffer, pos, find, call, span_cls, persistent_load_or_None, span_marker) -> (obj, end_pos)
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <string.h>

static PyObject *UnpicklingError;   /* pickle.UnpicklingError */

typedef struct {
    PyObject **v;
    Py_ssize_t n, cap;
} Stack;

typedef struct {
    Py_ssize_t *v;
    Py_ssize_t n, cap;
} Marks;

static int malformed(const char *what) {
    PyErr_Format(UnpicklingError, "malformed update payload: %s", what);
    return -1;
}

static int push(Stack *s, PyObject *o) {   /* steals o */
    if (o == NULL) return -1;
    if (s->n == s->cap) {
        Py_ssize_t cap = s->cap ? 2 * s->cap : 64;
        PyObject **v = PyMem_Realloc(s->v, (size_t)cap * sizeof(PyObject *));
        if (v == NULL) {
            Py_DECREF(o);
            PyErr_NoMemory();
            return -1;
        }
        s->v = v;
        s->cap = cap;
    }
    s->v[s->n++] = o;
    return 0;
}

static PyObject *pop(Stack *s) {           /* new reference owned by the caller */
    if (s->n == 0) {
        malformed("stack underflow");
        return NULL;
    }
    return s->v[--s->n];
}

static int mark_push(Marks *m, Py_ssize_t at) {
    if (m->n == m->cap) {
        Py_ssize_t cap = m->cap ? 2 * m->cap : 16;
        Py_ssize_t *v = PyMem_Realloc(m->v, (size_t)cap * sizeof(Py_ssize_t));
        if (v == NULL) {
            PyErr_NoMemory();
            return -1;
        }
        m->v = v;
        m->cap = cap;
    }
    m->v[m->n++] = at;
    return 0;
}

static Py_ssize_t mark_pop(Marks *m, const Stack *s) {
    if (m->n == 0) return malformed("MARK expected"), -1;
    Py_ssize_t k = m->v[--m->n];
    if (k > s->n) return malformed("stack underflow below MARK"), -1;
    return k;
}

/* stack[k:] as a new tuple / list; the items' references move into it */
static PyObject *take_tuple(Stack *s, Py_ssize_t k) {
    PyObject *t = PyTuple_New(s->n - k);
    if (t == NULL) return NULL;
    for (Py_ssize_t i = k; i < s->n; ++i) PyTuple_SET_ITEM(t, i - k, s->v[i]);
    s->n = k;
    return t;
}

static PyObject *take_list(Stack *s, Py_ssize_t k) {
    PyObject *t = PyList_New(s->n - k);
    if (t == NULL) return NULL;
    for (Py_ssize_t i = k; i < s->n; ++i) PyList_SET_ITEM(t, i - k, s->v[i]);
    s->n = k;
    return t;
}

static uint64_t le(const unsigned char *p, int n) {
    uint64_t v = 0;
    for (int i = n - 1; i >= 0; --i) v = (v << 8) | p[i];
    return v;
}

#define NEED(k)                                                             \
    do {                                                                    \
        if ((Py_ssize_t)(k) < 0 || p + (Py_ssize_t)(k) > n) {               \
            malformed("truncated");                                         \
            goto fail;                                                      \
        }                                                                   \
    } while (0)
#define TOP_OR_FAIL()                                                       \
    do {                                                                    \
        if (st.n == 0) {                                                    \
            malformed("stack underflow");                                   \
            goto fail;                                                      \
        }                                                                   \
    } while (0)
#define PUSH(o)                                                             \
    do {                                                                    \
        if (push(&st, (o)) < 0) goto fail;                                  \
    } while (0)

static PyObject *vm_load(PyObject *self, PyObject *args) {
    (void)self;
    PyObject *bufobj, *find, *call, *span_cls, *pload, *span_marker;
    Py_ssize_t p;
    if (!PyArg_ParseTuple(args, "OnOOOOO", &bufobj, &p, &find, &call, &span_cls, &pload, &span_marker)) return NULL;
    Py_buffer view;
    if (PyObject_GetBuffer(bufobj, &view, PyBUF_SIMPLE) < 0) return NULL;
    const unsigned char *b = (const unsigned char *)view.buf;
    const Py_ssize_t n = view.len;
    Stack st = {NULL, 0, 0};
    Marks mk = {NULL, 0, 0};
    PyObject *memo = PyDict_New();
    PyObject *result = NULL;
    if (memo == NULL) goto fail;
    if (p < 0) {
        malformed("negative start");
        goto fail;
    }
    for (;;) {
        NEED(1);
        const unsigned op = b[p++];
        switch (op) {
        case 0x94: {                                   /* MEMOIZE */
            TOP_OR_FAIL();
            PyObject *key = PyLong_FromSsize_t(PyDict_GET_SIZE(memo));
            if (key == NULL) goto fail;
            int rc = PyDict_SetItem(memo, key, st.v[st.n - 1]);
            Py_DECREF(key);
            if (rc < 0) goto fail;
            break;
        }
        case 0x4B:                                     /* BININT1 */
            NEED(1);
            PUSH(PyLong_FromLong(b[p]));
            p += 1;
            break;
        case 0x52:                                     /* REDUCE */
        case 0x81: {                                   /* NEWOBJ */
            PyObject *a = pop(&st);
            if (a == NULL) goto fail;
            if (st.n == 0) {
                Py_DECREF(a);
                malformed("stack underflow");
                goto fail;
            }
            PyObject *fn = st.v[st.n - 1];
            PyObject *r = PyObject_CallFunctionObjArgs(call, fn, a, NULL);
            Py_DECREF(a);
            if (r == NULL) goto fail;
            st.v[st.n - 1] = r;
            Py_DECREF(fn);
            break;
        }
        case 0x68:                                     /* BINGET */
        case 0x6A: {                                   /* LONG_BINGET */
            const int w = op == 0x68 ? 1 : 4;
            NEED(w);
            PyObject *key = PyLong_FromUnsignedLongLong(le(b + p, w));
            p += w;
            if (key == NULL) goto fail;
            PyObject *v = PyDict_GetItemWithError(memo, key);
            Py_DECREF(key);
            if (v == NULL) {
                if (!PyErr_Occurred()) malformed("memo key missing");
                goto fail;
            }
            Py_INCREF(v);
            PUSH(v);
            break;
        }
        case 0x71:                                     /* BINPUT */
        case 0x72: {                                   /* LONG_BINPUT */
            const int w = op == 0x71 ? 1 : 4;
            NEED(w);
            TOP_OR_FAIL();
            PyObject *key = PyLong_FromUnsignedLongLong(le(b + p, w));
            p += w;
            if (key == NULL) goto fail;
            int rc = PyDict_SetItem(memo, key, st.v[st.n - 1]);
            Py_DECREF(key);
            if (rc < 0) goto fail;
            break;
        }
        case 0x8C:                                     /* SHORT_BINUNICODE */
        case 0x58:                                     /* BINUNICODE */
        case 0x8D: {                                   /* BINUNICODE8 */
            const int w = op == 0x8C ? 1 : op == 0x58 ? 4 : 8;
            NEED(w);
            const uint64_t len = le(b + p, w);
            p += w;
            if (len > (uint64_t)(n - p)) {
                malformed("truncated");
                goto fail;
            }
            PUSH(PyUnicode_DecodeUTF8((const char *)b + p, (Py_ssize_t)len, "strict"));
            p += (Py_ssize_t)len;
            break;
        }
        case 0x43:                                     /* SHORT_BINBYTES */
        case 0x42:                                     /* BINBYTES */
        case 0x8E: {                                   /* BINBYTES8: a span, no copy */
            const int w = op == 0x43 ? 1 : op == 0x42 ? 4 : 8;
            NEED(w);
            const uint64_t len = le(b + p, w);
            p += w;
            if (len > (uint64_t)(n - p)) {
                malformed("truncated");
                goto fail;
            }
            if (st.n > 0 && st.v[st.n - 1] == span_marker)   /* torch.storage._load_from_bytes(...) */
                PUSH(PyObject_CallFunction(span_cls, "nn", p, (Py_ssize_t)len));
            else
                PUSH(PyBytes_FromStringAndSize((const char *)b + p, (Py_ssize_t)len));
            p += (Py_ssize_t)len;
            break;
        }
        case 0x96: {                                   /* BYTEARRAY8 (protocol 5) */
            NEED(8);
            const uint64_t len = le(b + p, 8);
            p += 8;
            if (len > (uint64_t)(n - p)) {
                malformed("truncated");
                goto fail;
            }
            PUSH(PyByteArray_FromStringAndSize((const char *)b + p, (Py_ssize_t)len));
            p += (Py_ssize_t)len;
            break;
        }
        case 0x85: {                                   /* TUPLE1 */
            TOP_OR_FAIL();
            PyObject *t = PyTuple_New(1);
            if (t == NULL) goto fail;
            PyTuple_SET_ITEM(t, 0, st.v[st.n - 1]);
            st.v[st.n - 1] = t;
            break;
        }
        case 0x86:                                     /* TUPLE2 */
        case 0x87: {                                   /* TUPLE3 */
            const Py_ssize_t k = op == 0x86 ? 2 : 3;
            if (st.n < k) {
                malformed("stack underflow");
                goto fail;
            }
            PUSH(take_tuple(&st, st.n - k));
            break;
        }
        case 0x28:                                     /* MARK */
            if (mark_push(&mk, st.n) < 0) goto fail;
            break;
        case 0x74:                                     /* TUPLE */
        case 0x6C: {                                   /* LIST */
            const Py_ssize_t k = mark_pop(&mk, &st);
            if (k < 0) goto fail;
            PUSH(op == 0x74 ? take_tuple(&st, k) : take_list(&st, k));
            break;
        }
        case 0x91: {                                   /* FROZENSET */
            const Py_ssize_t k = mark_pop(&mk, &st);
            if (k < 0) goto fail;
            PyObject *items = take_list(&st, k);
            if (items == NULL) goto fail;
            PyObject *fs = PyFrozenSet_New(items);
            Py_DECREF(items);
            PUSH(fs);
            break;
        }
        case 0x29:                                     /* EMPTY_TUPLE */
            PUSH(PyTuple_New(0));
            break;
        case 0x89:                                     /* NEWFALSE */
            Py_INCREF(Py_False);
            PUSH(Py_False);
            break;
        case 0x88:                                     /* NEWTRUE */
            Py_INCREF(Py_True);
            PUSH(Py_True);
            break;
        case 0x4E:                                     /* NONE */
            Py_INCREF(Py_None);
            PUSH(Py_None);
            break;
        case 0x80:                                     /* PROTO */
            NEED(1);
            p += 1;
            break;
        case 0x95:                                     /* FRAME (a hint: skipped) */
            NEED(8);
            p += 8;
            break;
        case 0x2E:                                     /* STOP */
            result = pop(&st);
            if (result == NULL) goto fail;
            goto done;
        case 0x7D:                                     /* EMPTY_DICT */
            PUSH(PyDict_New());
            break;
        case 0x5D:                                     /* EMPTY_LIST */
            PUSH(PyList_New(0));
            break;
        case 0x8F:                                     /* EMPTY_SET */
            PUSH(PySet_New(NULL));
            break;
        case 0x4D:                                     /* BININT2 */
            NEED(2);
            PUSH(PyLong_FromLong((long)le(b + p, 2)));
            p += 2;
            break;
        case 0x4A:                                     /* BININT */
            NEED(4);
            PUSH(PyLong_FromLong((long)(int32_t)(uint32_t)le(b + p, 4)));
            p += 4;
            break;
        case 0x8A: {                                   /* LONG1 */
            NEED(1);
            const Py_ssize_t len = b[p];
            p += 1;
            NEED(len);
            PUSH(_PyLong_FromByteArray(b + p, (size_t)len, /*little_endian=*/1, /*is_signed=*/1));
            p += len;
            break;
        }
        case 0x47: {                                   /* BINFLOAT (big-endian double) */
            NEED(8);
#if PY_VERSION_HEX >= 0x030B0000
            const double d = PyFloat_Unpack8((const char *)b + p, /*le=*/0);
#else
            const double d = _PyFloat_Unpack8(b + p, /*le=*/0);
#endif
            if (d == -1.0 && PyErr_Occurred()) goto fail;
            PUSH(PyFloat_FromDouble(d));
            p += 8;
            break;
        }
        case 0x65:                                     /* APPENDS */
        case 0x90: {                                   /* ADDITEMS */
            const Py_ssize_t k = mark_pop(&mk, &st);
            if (k < 0) goto fail;
            if (k == 0) {
                malformed("stack underflow");
                goto fail;
            }
            PyObject *items = take_list(&st, k);
            if (items == NULL) goto fail;
            PyObject *tgt = st.v[st.n - 1];
            PyObject *r;
            if (op == 0x65 && PyList_CheckExact(tgt)) {
                r = PyList_SetSlice(tgt, PY_SSIZE_T_MAX, PY_SSIZE_T_MAX, items) < 0 ? NULL : Py_NewRef(Py_None);
            } else {
                r = PyObject_CallMethod(tgt, op == 0x65 ? "extend" : "update", "O", items);
            }
            Py_DECREF(items);
            if (r == NULL) goto fail;
            Py_DECREF(r);
            break;
        }
        case 0x61: {                                   /* APPEND */
            PyObject *v = pop(&st);
            if (v == NULL) goto fail;
            if (st.n == 0) {
                Py_DECREF(v);
                malformed("stack underflow");
                goto fail;
            }
            PyObject *tgt = st.v[st.n - 1];
            int rc;
            if (PyList_CheckExact(tgt)) {
                rc = PyList_Append(tgt, v);
            } else {
                PyObject *r = PyObject_CallMethod(tgt, "append", "O", v);
                rc = r ? 0 : -1;
                Py_XDECREF(r);
            }
            Py_DECREF(v);
            if (rc < 0) goto fail;
            break;
        }
        case 0x75: {                                   /* SETITEMS */
            const Py_ssize_t k = mark_pop(&mk, &st);
            if (k < 0) goto fail;
            if (k == 0) {
                malformed("stack underflow");
                goto fail;
            }
            PyObject *d = st.v[k - 1];
            int rc = 0;
            Py_ssize_t i = k;
            for (; i + 1 < st.n && rc == 0; i += 2) rc = PyObject_SetItem(d, st.v[i], st.v[i + 1]);
            if (rc == 0 && i < st.n) {              /* an odd item: Python's items[i + 1] IndexError */
                malformed("odd SETITEMS");
                rc = -1;
            }
            for (Py_ssize_t j = k; j < st.n; ++j) Py_DECREF(st.v[j]);
            st.n = k;
            if (rc < 0) goto fail;
            break;
        }
        case 0x73: {                                   /* SETITEM */
            if (st.n < 3) {
                malformed("stack underflow");
                goto fail;
            }
            PyObject *v = st.v[st.n - 1], *key = st.v[st.n - 2];
            st.n -= 2;
            int rc = PyObject_SetItem(st.v[st.n - 1], key, v);
            Py_DECREF(v);
            Py_DECREF(key);
            if (rc < 0) goto fail;
            break;
        }
        case 0x93: {                                   /* STACK_GLOBAL */
            if (st.n < 2) {
                malformed("stack underflow");
                goto fail;
            }
            PyObject *name = st.v[st.n - 1], *module = st.v[st.n - 2];
            st.n -= 2;
            PyObject *g = PyObject_CallFunctionObjArgs(find, module, name, NULL);
            Py_DECREF(name);
            Py_DECREF(module);
            PUSH(g);
            break;
        }
        case 0x63: {                                   /* GLOBAL "module\nname\n" */
            Py_ssize_t lim = n - p < 256 ? n - p : 256;
            const unsigned char *e1 = memchr(b + p, '\n', (size_t)lim);
            if (e1 == NULL) {
                malformed("GLOBAL without newline");
                goto fail;
            }
            const Py_ssize_t l1 = e1 - (b + p), q = p + l1 + 1;
            lim = n - q < 256 ? n - q : 256;
            const unsigned char *e2 = lim > 0 ? memchr(b + q, '\n', (size_t)lim) : NULL;
            if (e2 == NULL) {
                malformed("GLOBAL without newline");
                goto fail;
            }
            const Py_ssize_t l2 = e2 - (b + q);
            PyObject *module = PyUnicode_DecodeUTF8((const char *)b + p, l1, "strict");
            PyObject *name = module ? PyUnicode_DecodeUTF8((const char *)b + q, l2, "strict") : NULL;
            p = q + l2 + 1;
            if (name == NULL) {
                Py_XDECREF(module);
                goto fail;
            }
            PyObject *g = PyObject_CallFunctionObjArgs(find, module, name, NULL);
            Py_DECREF(module);
            Py_DECREF(name);
            PUSH(g);
            break;
        }
        case 0x62: {                                   /* BUILD: only an empty state */
            PyObject *state = pop(&st);
            if (state == NULL) goto fail;
            const int t = PyObject_IsTrue(state);
            Py_DECREF(state);
            if (t < 0) goto fail;
            if (t) {
                PyErr_SetString(UnpicklingError, "BUILD with state is not allowed in update payloads");
                goto fail;
            }
            break;
        }
        case 0x51: {                                   /* BINPERSID */
            PyObject *pid = pop(&st);
            if (pid == NULL) goto fail;
            if (pload == Py_None) {
                Py_DECREF(pid);
                PyErr_SetString(UnpicklingError, "persistent id outside a storage stream");
                goto fail;
            }
            PyObject *r = PyObject_CallFunctionObjArgs(pload, pid, NULL);
            Py_DECREF(pid);
            PUSH(r);
            break;
        }
        default:
            PyErr_Format(UnpicklingError, "opcode 0x%02x not allowed in update payloads", op);
            goto fail;
        }
    }
done: {
    PyObject *out = Py_BuildValue("(Nn)", result, p);
    result = NULL;
    for (Py_ssize_t i = 0; i < st.n; ++i) Py_DECREF(st.v[i]);
    PyMem_Free(st.v);
    PyMem_Free(mk.v);
    Py_XDECREF(memo);
    PyBuffer_Release(&view);
    return out;
}
fail:
    for (Py_ssize_t i = 0; i < st.n; ++i) Py_DECREF(st.v[i]);
    PyMem_Free(st.v);
    PyMem_Free(mk.v);
    Py_XDECREF(memo);
    PyBuffer_Release(&view);
    return NULL;
}

/* storage_head(buffer, start, end, headers) -> (type_name, numel, data_pos) | None
 *
 * The start of a legacy torch.save stream of one storage (ingest._storage_from_span): one of
 * the already-validated stream headers (magic, protocol, sys-info pickles: `headers`, a list
 * of bytes), then torch's own storage record -- ('storage', torch.<T>Storage, key, location,
 * numel, None) as legacy _save writes it (protocol 2, BININT1/2/BININT count), the key list
 * [key] and the u64 element count -- every byte checked, all inside [start, end).  Returns
 * None when the stream departs from that layout in any byte; the caller then parses it with
 * the VM (ingest._parse_storage_record_slow and the persistent-id load). */
static int lit(const unsigned char *b, Py_ssize_t *p, Py_ssize_t end, const char *s, Py_ssize_t k) {
    if (*p + k > end || memcmp(b + *p, s, (size_t)k) != 0) return 0;
    *p += k;
    return 1;
}

static PyObject *storage_head(PyObject *self, PyObject *args) {
    (void)self;
    PyObject *bufobj, *headers;
    Py_ssize_t p, end;
    if (!PyArg_ParseTuple(args, "OnnO!", &bufobj, &p, &end, &PyList_Type, &headers)) return NULL;
    Py_buffer view;
    if (PyObject_GetBuffer(bufobj, &view, PyBUF_SIMPLE) < 0) return NULL;
    const unsigned char *b = (const unsigned char *)view.buf;
    PyObject *out = NULL;
    if (p < 0 || end > view.len || p > end) goto none;
    int hit = 0;
    for (Py_ssize_t i = 0; i < PyList_GET_SIZE(headers) && !hit; ++i) {
        PyObject *h = PyList_GET_ITEM(headers, i);
        if (!PyBytes_Check(h)) continue;
        hit = lit(b, &p, end, PyBytes_AS_STRING(h), PyBytes_GET_SIZE(h));
    }
    if (!hit) goto none;
    static const char rec0[] = "\x80\x02(X\x07\x00\x00\x00storageq\x00" "ctorch\n";
    if (!lit(b, &p, end, rec0, sizeof(rec0) - 1)) goto none;
    const Py_ssize_t name0 = p;
    while (p < end && p - name0 < 64 && b[p] != '\n') {
        const unsigned char c = b[p];
        if (!((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_')) goto none;
        ++p;
    }
    const Py_ssize_t name1 = p;
    if (name1 == name0 || !lit(b, &p, end, "\nq\x01X", 4)) goto none;
    if (p + 4 > end) goto none;
    const Py_ssize_t klen = (Py_ssize_t)le(b + p, 4);
    p += 4;
    if (klen > end - p) goto none;
    const Py_ssize_t key0 = p;
    p += klen;
    if (!lit(b, &p, end, "q\x02X", 3) || p + 4 > end) goto none;
    const Py_ssize_t llen = (Py_ssize_t)le(b + p, 4);
    p += 4;
    if (llen > end - p) goto none;
    p += llen;
    if (!lit(b, &p, end, "q\x03", 2) || p >= end) goto none;
    int64_t numel;
    const unsigned char op = b[p++];
    if (op == 'K' && p + 1 <= end) {
        numel = b[p];
        p += 1;
    } else if (op == 'M' && p + 2 <= end) {
        numel = (int64_t)le(b + p, 2);
        p += 2;
    } else if (op == 'J' && p + 4 <= end) {
        numel = (int32_t)(uint32_t)le(b + p, 4);
        p += 4;
    } else {
        goto none;
    }
    if (numel < 0 || !lit(b, &p, end, "Ntq\x04Q.\x80\x02]q\x00X", 12) || p + 4 > end) goto none;
    if ((Py_ssize_t)le(b + p, 4) != klen) goto none;
    p += 4;
    if (p + klen > end || memcmp(b + p, b + key0, (size_t)klen) != 0) goto none;
    p += klen;
    if (!lit(b, &p, end, "q\x01" "a.", 4) || p + 8 > end) goto none;
    if (le(b + p, 8) != (uint64_t)numel) goto none;
    p += 8;
    out = Py_BuildValue("(s#Ln)", (const char *)b + name0, name1 - name0, (long long)numel, p);
    PyBuffer_Release(&view);
    return out;
none:
    PyBuffer_Release(&view);
    Py_RETURN_NONE;
}

static PyMethodDef methods[] = {
    {"load", vm_load, METH_VARARGS,
     "load(buffer, pos, find, call, span_cls, persistent_load, span_marker) -> (obj, end): the restricted pickle VM"},
    {"storage_head", storage_head, METH_VARARGS,
     "storage_head(buffer, start, end, headers) -> (type_name, numel, data_pos) or None"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_pickle_vm", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__pickle_vm(void) {
    PyObject *pk = PyImport_ImportModule("pickle");
    if (pk == NULL) return NULL;
    UnpicklingError = PyObject_GetAttrString(pk, "UnpicklingError");
    Py_DECREF(pk);
    if (UnpicklingError == NULL) return NULL;
    return PyModule_Create(&module);
}
