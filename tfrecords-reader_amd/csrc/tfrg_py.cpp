// tfrg_py.cpp — CPython binding of the host decode of single records (tfr_reader/_tfrg_py).
//
// tfrg_host_decode (tfrg_cpu.cpp, compiled into this module: no device runtime is loaded for a
// host decode) followed by the construction of the reference's object graph in C: a dict
// key -> raw feature in the record's key order, each raw feature answering WhichOneof("kind") and
// exposing the kind-checked float_list / int64_list / bytes_list whose .value is a fresh list per
// access (cython/decoder.pyx:304-376). Built like the reference's own Cython module: a ctypes call
// and Python-level object building cost several microseconds per record, this costs about one.
// Also the C bases of the device path's Feature objects over a batch's columns (ColRec, ColAcc).
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <string.h>

#include "../../include/tfrg.h"

namespace {

const char* const kKindName[4] = {"", "bytes_list", "float_list", "int64_list"};

// ---- value list (decoder.pyx:352-376: BytesList / FloatList / Int64List)
struct ValueList {
  PyObject_HEAD
  PyObject* values;  // list
};

void vl_dealloc(ValueList* self) {
  Py_XDECREF(self->values);
  Py_TYPE(self)->tp_free((PyObject*)self);
}

PyObject* vl_value(ValueList* self, void*) {  // a fresh list per access, as the reference
  return PyList_GetSlice(self->values, 0, PyList_GET_SIZE(self->values));
}

PyObject* vl_item(ValueList* self, Py_ssize_t i) { return PySequence_GetItem(self->values, i); }
Py_ssize_t vl_len(ValueList* self) { return PyList_GET_SIZE(self->values); }

PyGetSetDef vl_getset[] = {{"value", (getter)vl_value, nullptr, nullptr, nullptr}, {nullptr}};
PySequenceMethods vl_seq = {};   // __getitem__ only (FloatList, Int64List)
PySequenceMethods vlb_seq = {};  // __getitem__ and __len__ (BytesList, decoder.pyx:359)

PyTypeObject ValueListType = {PyVarObject_HEAD_INIT(nullptr, 0)};
PyTypeObject BytesValueListType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// ---- raw feature (decoder.pyx:314-349: Feature with WhichOneof and the kind-checked lists)
struct RawFeature {
  PyObject_HEAD
  int kind;
  PyObject* values;  // list
};

void rf_dealloc(RawFeature* self) {
  Py_XDECREF(self->values);
  Py_TYPE(self)->tp_free((PyObject*)self);
}

PyObject* rf_which(RawFeature* self, PyObject*) { return PyUnicode_FromString(kKindName[self->kind]); }

PyObject* rf_list(RawFeature* self, int want, const char* msg) {
  if (self->kind != want) {
    PyErr_SetString(PyExc_Exception, msg);
    return nullptr;
  }
  ValueList* v = PyObject_New(ValueList, want == 1 ? &BytesValueListType : &ValueListType);
  if (!v) return nullptr;
  Py_INCREF(self->values);
  v->values = self->values;
  return (PyObject*)v;
}
PyObject* rf_float(RawFeature* self, void*) { return rf_list(self, 2, "Feature is not a float_list"); }
PyObject* rf_int64(RawFeature* self, void*) { return rf_list(self, 3, "Feature is not an int64_list"); }
PyObject* rf_bytes(RawFeature* self, void*) { return rf_list(self, 1, "Feature is not a bytes_list"); }
PyObject* rf_kind(RawFeature* self, void*) { return PyUnicode_FromString(kKindName[self->kind]); }

PyObject* rf_reduce(RawFeature* self, PyObject*) {  // pickles as raw_feature(kind, values)
  PyObject* mod = PyImport_ImportModule("tfr_reader._tfrg_py");
  if (!mod) return nullptr;
  PyObject* fn = PyObject_GetAttrString(mod, "raw_feature");
  Py_DECREF(mod);
  if (!fn) return nullptr;
  return Py_BuildValue("(N(iO))", fn, self->kind, self->values);
}

PyMethodDef rf_methods[] = {{"WhichOneof", (PyCFunction)rf_which, METH_O, nullptr},
                            {"__reduce__", (PyCFunction)rf_reduce, METH_NOARGS, nullptr},
                            {nullptr}};
PyGetSetDef rf_getset[] = {{"float_list", (getter)rf_float, nullptr, nullptr, nullptr},
                           {"int64_list", (getter)rf_int64, nullptr, nullptr, nullptr},
                           {"bytes_list", (getter)rf_bytes, nullptr, nullptr, nullptr},
                           {"kind", (getter)rf_kind, nullptr, nullptr, nullptr},
                           {nullptr}};
PyTypeObject RawFeatureType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// ---- the device path's Feature objects over a batch's columns (tfr_reader/hip.py _record_class):
// a record is (batch, record index, layout), f[key] an accessor over a slice [lo, hi) of the slot's
// cached Python value list, .value that slice (a fresh list, feature.py:40-55). Python subclasses add
// the reference classes as bases (Feature, Int64List / FloatList / BytesList).
struct ColAcc {
  PyObject_HEAD
  PyObject* vals;  // list (null only for an instance made from Python: empty)
  Py_ssize_t lo, hi;
};

void ca_dealloc(ColAcc* self) {
  Py_XDECREF(self->vals);
  Py_TYPE(self)->tp_free((PyObject*)self);
}

PyObject* ca_value(ColAcc* self, void*) {
  if (!self->vals) return PyList_New(0);
  return PyList_GetSlice(self->vals, self->lo, self->hi);
}

PyGetSetDef ca_getset[] = {{"value", (getter)ca_value, nullptr, nullptr, nullptr}, {nullptr}};
PyTypeObject ColAccType = {PyVarObject_HEAD_INIT(nullptr, 0)};

struct ColRec {
  PyObject_HEAD
  PyObject* batch;  // BatchResult
  PyObject* cols;   // batch._py: per slot None or (values list, row splits list)
  PyObject* lay;    // _Layout
  PyObject* acc;    // lay.acc: key -> (slot, accessor class)
  PyObject* keys;   // lay.keys
  Py_ssize_t i;
};

void cr_dealloc(ColRec* self) {
  Py_XDECREF(self->batch);
  Py_XDECREF(self->cols);
  Py_XDECREF(self->lay);
  Py_XDECREF(self->acc);
  Py_XDECREF(self->keys);
  Py_TYPE(self)->tp_free((PyObject*)self);
}

// f[key]: the accessor of key's slot over record i's slice (feature.py:100-110); a missing key raises
// the reference's KeyError (feature.py:101-104)
PyObject* cr_subscript(ColRec* self, PyObject* key) {
  if (!self->acc) {
    PyErr_SetString(PyExc_TypeError, "uninitialised Feature");
    return nullptr;
  }
  PyObject* ent = PyDict_GetItemWithError(self->acc, key);
  if (!ent) {
    if (PyErr_Occurred()) return nullptr;
    PyObject* msg = PyUnicode_FromFormat("Feature '%S' not found in the example, expected one of %R", key, self->keys);
    if (msg) {
      PyErr_SetObject(PyExc_KeyError, msg);
      Py_DECREF(msg);
    }
    return nullptr;
  }
  const Py_ssize_t s = PyLong_AsSsize_t(PyTuple_GET_ITEM(ent, 0));
  if (s < 0 || s >= PyList_GET_SIZE(self->cols)) {
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_IndexError, "slot out of range");
    return nullptr;
  }
  PyObject* col = PyList_GET_ITEM(self->cols, s);
  PyObject* owned = nullptr;
  if (col == Py_None) {  // the slot's values as Python objects, converted once per batch
    owned = col = PyObject_CallMethod(self->batch, "_pycol", "n", s);
    if (!col) return nullptr;
  }
  PyObject* rs = PyTuple_GET_ITEM(col, 1);
  PyObject* vals = PyTuple_GET_ITEM(col, 0);
  Py_ssize_t lo = 0, hi = 0;
  if (self->i + 1 < PyList_GET_SIZE(rs)) {
    lo = PyLong_AsSsize_t(PyList_GET_ITEM(rs, self->i));
    hi = PyLong_AsSsize_t(PyList_GET_ITEM(rs, self->i + 1));
  }
  PyTypeObject* cls = (PyTypeObject*)PyTuple_GET_ITEM(ent, 1);
  ColAcc* a = (ColAcc*)cls->tp_alloc(cls, 0);
  if (a) {
    Py_INCREF(vals);
    a->vals = vals;
    a->lo = lo;
    a->hi = hi;
  }
  Py_XDECREF(owned);
  return (PyObject*)a;
}

Py_ssize_t cr_len(ColRec* self) { return self->keys ? PyList_GET_SIZE(self->keys) : 0; }

PyObject* cr_fields_names(ColRec* self, void*) {
  if (!self->keys) return PyList_New(0);
  return PyList_GetSlice(self->keys, 0, PyList_GET_SIZE(self->keys));
}
PyObject* cr_batch(ColRec* self, void*) { return Py_NewRef(self->batch ? self->batch : Py_None); }
PyObject* cr_lay(ColRec* self, void*) { return Py_NewRef(self->lay ? self->lay : Py_None); }
PyObject* cr_index(ColRec* self, void*) { return PyLong_FromSsize_t(self->i); }

PyMappingMethods cr_map = {(lenfunc)cr_len, (binaryfunc)cr_subscript, nullptr};
PyGetSetDef cr_getset[] = {{"fields_names", (getter)cr_fields_names, nullptr, nullptr, nullptr},
                           {"_batch", (getter)cr_batch, nullptr, nullptr, nullptr},
                           {"_lay", (getter)cr_lay, nullptr, nullptr, nullptr},
                           {"_i", (getter)cr_index, nullptr, nullptr, nullptr},
                           {nullptr}};
PyTypeObject ColRecType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// make_records(cls, batch, cols, start, inv, layouts) -> [cls record] for records start + j, j <
// len(inv), record start + j having layout layouts[inv[j]] (inv: int64 buffer)
PyObject* py_make_records(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 6 || !PyType_Check(args[0]) || !PyType_IsSubtype((PyTypeObject*)args[0], &ColRecType) ||
      !PyList_Check(args[2]) || !PyList_Check(args[5])) {
    PyErr_SetString(PyExc_TypeError, "make_records(cls, batch, cols: list, start: int, inv: int64 buffer, layouts: list)");
    return nullptr;
  }
  PyTypeObject* cls = (PyTypeObject*)args[0];
  const Py_ssize_t start = PyLong_AsSsize_t(args[3]);
  if (start < 0) {
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "start < 0");
    return nullptr;
  }
  Py_buffer vb;
  if (PyObject_GetBuffer(args[4], &vb, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) < 0) return nullptr;
  PyObject* out = nullptr;
  const Py_ssize_t nl = PyList_GET_SIZE(args[5]);
  PyObject** acc = nullptr;
  PyObject** keys = nullptr;
  if (vb.itemsize != 8 || !vb.format || (vb.format[0] != 'q' && vb.format[0] != 'l')) {
    PyErr_SetString(PyExc_TypeError, "inv must be an int64 buffer");
    goto done;
  }
  acc = (PyObject**)PyMem_Calloc(nl ? nl : 1, sizeof(PyObject*));
  keys = (PyObject**)PyMem_Calloc(nl ? nl : 1, sizeof(PyObject*));
  if (!acc || !keys) {
    PyErr_NoMemory();
    goto done;
  }
  for (Py_ssize_t l = 0; l < nl; ++l) {
    acc[l] = PyObject_GetAttrString(PyList_GET_ITEM(args[5], l), "acc");
    keys[l] = acc[l] ? PyObject_GetAttrString(PyList_GET_ITEM(args[5], l), "keys") : nullptr;
    if (!keys[l]) goto done;
    if (!PyDict_Check(acc[l]) || !PyList_Check(keys[l])) {
      PyErr_SetString(PyExc_TypeError, "layout.acc must be a dict and layout.keys a list");
      goto done;
    }
  }
  {
    const int64_t* inv = (const int64_t*)vb.buf;
    const Py_ssize_t n = vb.len / 8;
    out = PyList_New(n);
    if (!out) goto done;
    for (Py_ssize_t j = 0; j < n; ++j) {
      const int64_t l = inv[j];
      if (l < 0 || l >= nl) {
        PyErr_SetString(PyExc_IndexError, "layout index out of range");
        Py_CLEAR(out);
        goto done;
      }
      ColRec* r = (ColRec*)cls->tp_alloc(cls, 0);
      if (!r) {
        Py_CLEAR(out);
        goto done;
      }
      r->batch = Py_NewRef(args[1]);
      r->cols = Py_NewRef(args[2]);
      r->lay = Py_NewRef(PyList_GET_ITEM(args[5], l));
      r->acc = Py_NewRef(acc[l]);
      r->keys = Py_NewRef(keys[l]);
      r->i = start + j;
      PyList_SET_ITEM(out, j, (PyObject*)r);
    }
  }
done:
  if (acc)
    for (Py_ssize_t l = 0; l < nl; ++l) {
      Py_XDECREF(acc[l]);
      Py_XDECREF(keys[l]);
    }
  PyMem_Free(acc);
  PyMem_Free(keys);
  PyBuffer_Release(&vb);
  return out;
}

// ---- a host-decoded record as the reference's Feature (feature.py:69-110) over its key -> raw feature
// dict: f[key] makes the accessor (the ColAcc subclass of the key's kind over the raw feature's value
// list) in C. Python subclass: tfr_reader/host.py.
struct HostRec {
  PyObject_HEAD
  PyObject* dict;
};

PyTypeObject* g_acc[4] = {nullptr, nullptr, nullptr, nullptr};  // accessor class per kind (set_accessors)
PyTypeObject* g_host_cls = nullptr;                               // HostRec subclass (set_accessors)

void hr_dealloc(HostRec* self) {
  Py_XDECREF(self->dict);
  Py_TYPE(self)->tp_free((PyObject*)self);
}

PyObject* hr_subscript(HostRec* self, PyObject* key) {
  if (!self->dict) {
    PyErr_SetString(PyExc_TypeError, "uninitialised Feature");
    return nullptr;
  }
  PyObject* raw = PyDict_GetItemWithError(self->dict, key);
  if (!raw) {
    if (PyErr_Occurred()) return nullptr;
    PyObject* keys = PyDict_Keys(self->dict);
    if (!keys) return nullptr;
    PyObject* msg = PyUnicode_FromFormat("Feature '%S' not found in the example, expected one of %R", key, keys);
    Py_DECREF(keys);
    if (msg) {
      PyErr_SetObject(PyExc_KeyError, msg);
      Py_DECREF(msg);
    }
    return nullptr;
  }
  if (Py_TYPE(raw) != &RawFeatureType) {
    PyErr_SetString(PyExc_TypeError, "not a raw feature of the host decode");
    return nullptr;
  }
  RawFeature* rf = (RawFeature*)raw;
  PyTypeObject* cls = g_acc[rf->kind];
  if (!cls) {
    PyErr_SetString(PyExc_RuntimeError, "set_accessors() was not called");
    return nullptr;
  }
  ColAcc* a = (ColAcc*)cls->tp_alloc(cls, 0);
  if (!a) return nullptr;
  Py_INCREF(rf->values);
  a->vals = rf->values;
  a->lo = 0;
  a->hi = PyList_GET_SIZE(rf->values);
  return (PyObject*)a;
}

Py_ssize_t hr_len(HostRec* self) { return self->dict ? PyDict_GET_SIZE(self->dict) : 0; }
PyObject* hr_feature(HostRec* self, void*) { return Py_NewRef(self->dict ? self->dict : Py_None); }
PyObject* hr_fields_names(HostRec* self, void*) { return self->dict ? PyDict_Keys(self->dict) : PyList_New(0); }

PyMappingMethods hr_map = {(lenfunc)hr_len, (binaryfunc)hr_subscript, nullptr};
PyGetSetDef hr_getset[] = {{"feature", (getter)hr_feature, nullptr, nullptr, nullptr},
                           {"fields_names", (getter)hr_fields_names, nullptr, nullptr, nullptr},
                           {nullptr}};
PyTypeObject HostRecType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// set_accessors(host_cls, bytes_acc, float_acc, int64_acc): the Python classes the C paths create
PyObject* py_set_accessors(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 4 || !PyType_Check(args[0]) || !PyType_IsSubtype((PyTypeObject*)args[0], &HostRecType)) {
    PyErr_SetString(PyExc_TypeError, "set_accessors(host_cls, bytes_acc, float_acc, int64_acc)");
    return nullptr;
  }
  for (int k = 1; k <= 3; ++k)
    if (!PyType_Check(args[k]) || !PyType_IsSubtype((PyTypeObject*)args[k], &ColAccType)) {
      PyErr_SetString(PyExc_TypeError, "accessor classes must subclass ColAcc");
      return nullptr;
    }
  Py_XSETREF(g_host_cls, (PyTypeObject*)Py_NewRef(args[0]));
  for (int k = 1; k <= 3; ++k) Py_XSETREF(g_acc[k], (PyTypeObject*)Py_NewRef(args[k]));
  Py_RETURN_NONE;
}

// split_bytes(buf, off, len) -> [bytes(buf[off[j]:off[j] + len[j]])] (off, len: int64 buffers): a
// bytes_list column's elements as Python bytes, copied straight from the batch's buffer
PyObject* py_split_bytes(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 3) {
    PyErr_SetString(PyExc_TypeError, "split_bytes(buf, off: int64 buffer, len: int64 buffer)");
    return nullptr;
  }
  Py_buffer b, ob, lb;
  if (PyObject_GetBuffer(args[0], &b, PyBUF_C_CONTIGUOUS) < 0) return nullptr;
  if (PyObject_GetBuffer(args[1], &ob, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) < 0) {
    PyBuffer_Release(&b);
    return nullptr;
  }
  if (PyObject_GetBuffer(args[2], &lb, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) < 0) {
    PyBuffer_Release(&ob);
    PyBuffer_Release(&b);
    return nullptr;
  }
  PyObject* out = nullptr;
  auto i64 = [](const Py_buffer& v) { return v.itemsize == 8 && v.format && (v.format[0] == 'q' || v.format[0] == 'l'); };
  if (!i64(ob) || !i64(lb) || ob.len != lb.len) {
    PyErr_SetString(PyExc_TypeError, "off and len must be int64 buffers of one length");
  } else {
    const int64_t* o = (const int64_t*)ob.buf;
    const int64_t* l = (const int64_t*)lb.buf;
    const Py_ssize_t n = ob.len / 8;
    const char* p = (const char*)b.buf;
    out = PyList_New(n);
    for (Py_ssize_t j = 0; out && j < n; ++j) {
      if (o[j] < 0 || l[j] < 0 || o[j] > b.len || l[j] > b.len - o[j]) {
        PyErr_SetString(PyExc_IndexError, "bytes element outside the buffer");
        Py_CLEAR(out);
        break;
      }
      PyObject* x = PyBytes_FromStringAndSize(p + o[j], l[j]);
      if (!x) {
        Py_CLEAR(out);
        break;
      }
      PyList_SET_ITEM(out, j, x);
    }
  }
  PyBuffer_Release(&lb);
  PyBuffer_Release(&ob);
  PyBuffer_Release(&b);
  return out;
}

// one host context per thread (its result arrays are reused call after call)
struct TlsCtx {
  tfrg_host_ctx* c = nullptr;
  ~TlsCtx() {
    if (c) tfrg_host_ctx_destroy(c);
  }
};
thread_local TlsCtx tls;

PyObject* values_of(const tfrg_host_record& r, uint32_t e, const char* raw) {
  const uint32_t a = r.val_off[e], m = r.val_cnt[e];
  PyObject* list = PyList_New(m);
  if (!list) return nullptr;
  for (uint32_t j = 0; j < m; ++j) {
    PyObject* x;
    if (r.kind[e] == 3) {
      x = PyLong_FromLongLong(r.i64[a + j]);
    } else if (r.kind[e] == 2) {
      float f;
      memcpy(&f, &r.f32[a + j], 4);
      x = PyFloat_FromDouble((double)f);  // (float32 -> double, as the reference's vector<float>)
    } else {
      x = PyBytes_FromStringAndSize(raw + r.b_off[a + j], r.b_len[a + j]);
    }
    if (!x) {
      Py_DECREF(list);
      return nullptr;
    }
    PyList_SET_ITEM(list, j, x);
  }
  return list;
}

// decode(raw: bytes, flags: int) -> dict (key -> raw feature) | (status, aux) for a failing record
PyObject* decode_impl(PyObject* rawobj, PyObject* flagobj) {
  const char* raw = PyBytes_AS_STRING(rawobj);
  const Py_ssize_t len = PyBytes_GET_SIZE(rawobj);
  const unsigned long flags = PyLong_AsUnsignedLong(flagobj);
  if (PyErr_Occurred()) return nullptr;
  if (!tls.c && tfrg_host_ctx_create(&tls.c) != 0) return PyErr_NoMemory();
  tfrg_host_record r;
  const int rc = tfrg_host_decode(tls.c, (const uint8_t*)raw, (uint64_t)len, (uint32_t)flags, &r);
  if (rc != 0) {
    PyErr_Format(PyExc_RuntimeError, "tfrg_host_decode failed (%d)", rc);
    return nullptr;
  }
  if (r.status != 0) return Py_BuildValue("(iL)", r.status, (long long)r.aux);
  PyObject* d = PyDict_New();
  if (!d) return nullptr;
  for (uint32_t e = 0; e < r.n_entries; ++e) {
    PyObject* key = PyUnicode_DecodeUTF8(raw + r.key_off[e], r.key_len[e], "strict");
    PyObject* vals = key ? values_of(r, e, raw) : nullptr;
    RawFeature* f = vals ? PyObject_New(RawFeature, &RawFeatureType) : nullptr;
    if (!f) {
      Py_XDECREF(key);
      Py_XDECREF(vals);
      Py_DECREF(d);
      return nullptr;
    }
    f->kind = r.kind[e];
    f->values = vals;
    const int bad = PyDict_SetItem(d, key, (PyObject*)f);
    Py_DECREF(key);
    Py_DECREF(f);
    if (bad) {
      Py_DECREF(d);
      return nullptr;
    }
  }
  return d;
}

PyObject* py_decode(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 2 || !PyBytes_Check(args[0])) {
    PyErr_SetString(PyExc_TypeError, "decode(raw: bytes, flags: int)");
    return nullptr;
  }
  return decode_impl(args[0], args[1]);
}

// decode_feature(raw: bytes, flags: int) -> Feature (the set_accessors host class) | (status, aux)
PyObject* py_decode_feature(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 2 || !PyBytes_Check(args[0])) {
    PyErr_SetString(PyExc_TypeError, "decode_feature(raw: bytes, flags: int)");
    return nullptr;
  }
  if (!g_host_cls) {
    PyErr_SetString(PyExc_RuntimeError, "set_accessors() was not called");
    return nullptr;
  }
  PyObject* d = decode_impl(args[0], args[1]);
  if (!d || !PyDict_Check(d)) return d;
  HostRec* f = (HostRec*)g_host_cls->tp_alloc(g_host_cls, 0);
  if (!f) {
    Py_DECREF(d);
    return nullptr;
  }
  f->dict = d;
  return (PyObject*)f;
}

// raw_feature(kind: int, values: list) -> raw feature (the device path's records pickled, and tests)
PyObject* py_raw_feature(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 2 || !PyList_Check(args[1])) {
    PyErr_SetString(PyExc_TypeError, "raw_feature(kind: int, values: list)");
    return nullptr;
  }
  const long k = PyLong_AsLong(args[0]);
  if (k < 1 || k > 3) {
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "kind must be 1, 2 or 3");
    return nullptr;
  }
  RawFeature* f = PyObject_New(RawFeature, &RawFeatureType);
  if (!f) return nullptr;
  f->kind = (int)k;
  Py_INCREF(args[1]);
  f->values = args[1];
  return (PyObject*)f;
}

PyMethodDef methods[] = {{"decode", (PyCFunction)(void (*)(void))py_decode, METH_FASTCALL, nullptr},
                         {"raw_feature", (PyCFunction)(void (*)(void))py_raw_feature, METH_FASTCALL, nullptr},
                         {"make_records", (PyCFunction)(void (*)(void))py_make_records, METH_FASTCALL, nullptr},
                         {"split_bytes", (PyCFunction)(void (*)(void))py_split_bytes, METH_FASTCALL, nullptr},
                         {"set_accessors", (PyCFunction)(void (*)(void))py_set_accessors, METH_FASTCALL, nullptr},
                         {"decode_feature", (PyCFunction)(void (*)(void))py_decode_feature, METH_FASTCALL, nullptr},
                         {nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_tfrg_py", nullptr, -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__tfrg_py(void) {
  vl_seq.sq_item = (ssizeargfunc)vl_item;
  vlb_seq.sq_item = (ssizeargfunc)vl_item;
  vlb_seq.sq_length = (lenfunc)vl_len;
  ValueListType.tp_name = "tfr_reader._tfrg_py.ValueList";
  ValueListType.tp_basicsize = sizeof(ValueList);
  ValueListType.tp_dealloc = (destructor)vl_dealloc;
  ValueListType.tp_flags = Py_TPFLAGS_DEFAULT;
  ValueListType.tp_getset = vl_getset;
  ValueListType.tp_as_sequence = &vl_seq;
  BytesValueListType = ValueListType;
  BytesValueListType.tp_name = "tfr_reader._tfrg_py.BytesValueList";
  BytesValueListType.tp_as_sequence = &vlb_seq;
  RawFeatureType.tp_name = "tfr_reader._tfrg_py.RawFeature";
  RawFeatureType.tp_basicsize = sizeof(RawFeature);
  RawFeatureType.tp_dealloc = (destructor)rf_dealloc;
  RawFeatureType.tp_flags = Py_TPFLAGS_DEFAULT;
  RawFeatureType.tp_methods = rf_methods;
  RawFeatureType.tp_getset = rf_getset;
  ColAccType.tp_name = "tfr_reader._tfrg_py.ColAcc";
  ColAccType.tp_basicsize = sizeof(ColAcc);
  ColAccType.tp_dealloc = (destructor)ca_dealloc;
  ColAccType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_BASETYPE;
  ColAccType.tp_getset = ca_getset;
  ColRecType.tp_name = "tfr_reader._tfrg_py.ColRec";
  ColRecType.tp_basicsize = sizeof(ColRec);
  ColRecType.tp_dealloc = (destructor)cr_dealloc;
  ColRecType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_BASETYPE;
  ColRecType.tp_getset = cr_getset;
  ColRecType.tp_as_mapping = &cr_map;
  HostRecType.tp_name = "tfr_reader._tfrg_py.HostRec";
  HostRecType.tp_basicsize = sizeof(HostRec);
  HostRecType.tp_dealloc = (destructor)hr_dealloc;
  HostRecType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_BASETYPE;
  HostRecType.tp_getset = hr_getset;
  HostRecType.tp_as_mapping = &hr_map;
  if (PyType_Ready(&ValueListType) < 0 || PyType_Ready(&BytesValueListType) < 0 || PyType_Ready(&RawFeatureType) < 0 ||
      PyType_Ready(&ColAccType) < 0 || PyType_Ready(&ColRecType) < 0 || PyType_Ready(&HostRecType) < 0)
    return nullptr;
  PyObject* m = PyModule_Create(&module);
  if (!m) return nullptr;
  PyTypeObject* types[] = {&RawFeatureType, &ColAccType, &ColRecType, &HostRecType};
  const char* names[] = {"RawFeature", "ColAcc", "ColRec", "HostRec"};
  for (int t = 0; t < 4; ++t) {
    Py_INCREF(types[t]);
    if (PyModule_AddObject(m, names[t], (PyObject*)types[t]) < 0) {
      Py_DECREF(types[t]);
      Py_DECREF(m);
      return nullptr;
    }
  }
  return m;
}
