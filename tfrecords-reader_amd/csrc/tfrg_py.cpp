// tfrg_py.cpp — CPython binding of the host decode of single records (tfr_reader/_tfrg_py).
//
// tfrg_host_decode (tfrg_cpu.cpp, compiled into this module: no device runtime is loaded for a
// host decode) followed by the construction of the reference's object graph in C: a dict
// key -> raw feature in the record's key order, each raw feature answering WhichOneof("kind") and
// exposing the kind-checked float_list / int64_list / bytes_list whose .value is a fresh list per
// access (cython/decoder.pyx:304-376). Built like the reference's own Cython module: a ctypes call
// and Python-level object building cost several microseconds per record, this costs about one.
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
PyObject* py_decode(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 2 || !PyBytes_Check(args[0])) {
    PyErr_SetString(PyExc_TypeError, "decode(raw: bytes, flags: int)");
    return nullptr;
  }
  const char* raw = PyBytes_AS_STRING(args[0]);
  const Py_ssize_t len = PyBytes_GET_SIZE(args[0]);
  const unsigned long flags = PyLong_AsUnsignedLong(args[1]);
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
  if (PyType_Ready(&ValueListType) < 0 || PyType_Ready(&BytesValueListType) < 0 || PyType_Ready(&RawFeatureType) < 0)
    return nullptr;
  PyObject* m = PyModule_Create(&module);
  if (!m) return nullptr;
  Py_INCREF(&RawFeatureType);
  if (PyModule_AddObject(m, "RawFeature", (PyObject*)&RawFeatureType) < 0) {
    Py_DECREF(&RawFeatureType);
    Py_DECREF(m);
    return nullptr;
  }
  return m;
}
