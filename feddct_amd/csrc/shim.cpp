// shim.cpp — _fa_shim: the drop-in's per-call host bookkeeping in C++.
//
// Every server_aggregate call re-checks that each bound module still keeps
// its state in its arena (a parameter may have been replaced, or its .data
// swapped by model.to()/.data =), and after the kernel has written the
// buckets it bumps every bound tensor's autograd version counter, as the
// reference's load_state_dict (an in-place copy_) does.  Over the 21 modules
// of a 20-client wrn16_8 round that is 2,058 tensors; in Python it costs
// ~180 us before the launch.  Same semantics here, one C
// loop per module.  Host code only (no device work); built by
// feddct_amd/build.py against the running torch.
#include <Python.h>

#include <cstdint>
#include <cstring>

#include <torch/csrc/autograd/python_variable.h>
#include <torch/csrc/autograd/variable.h>

namespace {

// valid_views(dicts, names, tensors, ptrs) -> bool
//   dicts/names/tensors: equal-length tuples; ptrs: bytes of uint64 data
//   pointers.  True iff for every i: dicts[i][names[i]] is tensors[i] and
//   tensors[i].data_ptr() == ptrs[i].
PyObject* valid_views(PyObject*, PyObject* args) {
  PyObject *dicts, *names, *tensors, *ptrs;
  if (!PyArg_ParseTuple(args, "O!O!O!S", &PyTuple_Type, &dicts, &PyTuple_Type, &names,
                        &PyTuple_Type, &tensors, &ptrs))
    return nullptr;
  const Py_ssize_t n = PyTuple_GET_SIZE(tensors);
  if (PyTuple_GET_SIZE(dicts) != n || PyTuple_GET_SIZE(names) != n ||
      PyBytes_GET_SIZE(ptrs) != n * (Py_ssize_t)sizeof(uint64_t)) {
    PyErr_SetString(PyExc_ValueError, "valid_views: length mismatch");
    return nullptr;
  }
  const char* p = PyBytes_AS_STRING(ptrs);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* d = PyTuple_GET_ITEM(dicts, i);
    PyObject* t = PyTuple_GET_ITEM(tensors, i);
    if (!PyDict_Check(d)) {
      PyErr_SetString(PyExc_TypeError, "valid_views: dicts must hold dicts");
      return nullptr;
    }
    PyObject* cur = PyDict_GetItemWithError(d, PyTuple_GET_ITEM(names, i));  // borrowed
    if (cur == nullptr) {
      if (PyErr_Occurred()) return nullptr;
      Py_RETURN_FALSE;
    }
    if (cur != t || !THPVariable_Check(t)) Py_RETURN_FALSE;
    uint64_t want;
    std::memcpy(&want, p + i * sizeof(uint64_t), sizeof want);
    if ((uint64_t)(uintptr_t)THPVariable_Unpack(t).data_ptr() != want) Py_RETURN_FALSE;
  }
  Py_RETURN_TRUE;
}

// The round fast path's check (r04): a dict's version tag (PEP 509; CPython
// < 3.12 keeps it in every dict) changes with every store into the dict, so
// an unchanged tag proves that each parameter / buffer slot still holds the
// tensor bound to it, and only the `.data` swap (which leaves the dict alone)
// remains to be checked, one data pointer per tensor — no dict lookups.
// dict_tags(dicts) -> bytes of uint64 tags, or None where tags are not
// available (the caller then keeps the lookup check).
// valid_tagged(dicts, tags, tensors, ptrs) -> bool: every dict's tag
// unchanged and every tensor's data pointer the bound one.
#if PY_VERSION_HEX < 0x030C0000
#define FA_DICT_TAGS 1
#endif

PyObject* dict_tags(PyObject*, PyObject* args) {
  PyObject* dicts;
  if (!PyArg_ParseTuple(args, "O!", &PyTuple_Type, &dicts)) return nullptr;
#ifdef FA_DICT_TAGS
  const Py_ssize_t n = PyTuple_GET_SIZE(dicts);
  PyObject* out = PyBytes_FromStringAndSize(nullptr, n * (Py_ssize_t)sizeof(uint64_t));
  if (!out) return nullptr;
  char* p = PyBytes_AS_STRING(out);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* d = PyTuple_GET_ITEM(dicts, i);
    if (!PyDict_Check(d)) {
      Py_DECREF(out);
      PyErr_SetString(PyExc_TypeError, "dict_tags: expected dicts");
      return nullptr;
    }
    const uint64_t tag = ((PyDictObject*)d)->ma_version_tag;
    std::memcpy(p + i * sizeof(uint64_t), &tag, sizeof tag);
  }
  return out;
#else
  (void)dicts;
  Py_RETURN_NONE;
#endif
}

PyObject* valid_tagged(PyObject*, PyObject* args) {
  PyObject *dicts, *tags, *tensors, *ptrs;
  if (!PyArg_ParseTuple(args, "O!SO!S", &PyTuple_Type, &dicts, &tags, &PyTuple_Type, &tensors,
                        &ptrs))
    return nullptr;
#ifdef FA_DICT_TAGS
  const Py_ssize_t nd = PyTuple_GET_SIZE(dicts), n = PyTuple_GET_SIZE(tensors);
  if (PyBytes_GET_SIZE(tags) != nd * (Py_ssize_t)sizeof(uint64_t) ||
      PyBytes_GET_SIZE(ptrs) != n * (Py_ssize_t)sizeof(uint64_t)) {
    PyErr_SetString(PyExc_ValueError, "valid_tagged: length mismatch");
    return nullptr;
  }
  const char* tp = PyBytes_AS_STRING(tags);
  for (Py_ssize_t i = 0; i < nd; ++i) {
    PyObject* d = PyTuple_GET_ITEM(dicts, i);
    uint64_t want;
    std::memcpy(&want, tp + i * sizeof(uint64_t), sizeof want);
    if (!PyDict_Check(d) || ((PyDictObject*)d)->ma_version_tag != want) Py_RETURN_FALSE;
  }
  const char* p = PyBytes_AS_STRING(ptrs);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* t = PyTuple_GET_ITEM(tensors, i);
    if (!THPVariable_Check(t)) Py_RETURN_FALSE;
    uint64_t want;
    std::memcpy(&want, p + i * sizeof(uint64_t), sizeof want);
    if ((uint64_t)(uintptr_t)THPVariable_Unpack(t).data_ptr() != want) Py_RETURN_FALSE;
  }
  Py_RETURN_TRUE;
#else
  (void)dicts;
  (void)tags;
  (void)tensors;
  (void)ptrs;
  Py_RETURN_FALSE;
#endif
}

// bump_versions(tensors) -> None: torch.autograd.graph.increment_version
// for every tensor of the tuple.
PyObject* bump_versions(PyObject*, PyObject* args) {
  PyObject* tensors;
  if (!PyArg_ParseTuple(args, "O!", &PyTuple_Type, &tensors)) return nullptr;
  const Py_ssize_t n = PyTuple_GET_SIZE(tensors);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* t = PyTuple_GET_ITEM(tensors, i);
    if (!THPVariable_Check(t)) {
      PyErr_SetString(PyExc_TypeError, "bump_versions: expected tensors");
      return nullptr;
    }
    const at::Tensor& x = THPVariable_Unpack(t);
    if (!x.is_inference()) torch::autograd::impl::bump_version(x);
  }
  Py_RETURN_NONE;
}

// grad_state(params, views) -> 0: every params[i].grad is views[i] (the flat
// gradient bucket is bound); 1: every .grad is None; 2: anything else.
PyObject* grad_state(PyObject*, PyObject* args) {
  PyObject *params, *views;
  if (!PyArg_ParseTuple(args, "O!O!", &PyTuple_Type, &params, &PyTuple_Type, &views))
    return nullptr;
  const Py_ssize_t n = PyTuple_GET_SIZE(params);
  if (PyTuple_GET_SIZE(views) != n) {
    PyErr_SetString(PyExc_ValueError, "grad_state: length mismatch");
    return nullptr;
  }
  bool bound = true, none = true;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* t = PyTuple_GET_ITEM(params, i);
    PyObject* v = PyTuple_GET_ITEM(views, i);
    if (!THPVariable_Check(t) || !THPVariable_Check(v)) {
      PyErr_SetString(PyExc_TypeError, "grad_state: expected tensors");
      return nullptr;
    }
    const at::Tensor& g = THPVariable_Unpack(t).grad();
    if (g.defined()) none = false;
    if (!g.defined() || g.unsafeGetTensorImpl() != THPVariable_Unpack(v).unsafeGetTensorImpl())
      bound = false;
  }
  return PyLong_FromLong(bound ? 0 : (none ? 1 : 2));
}

// bind_grads(params, views) -> None: params[i].grad = views[i] (leaf
// parameters; the views are slices of one flat gradient bucket).
PyObject* bind_grads(PyObject*, PyObject* args) {
  PyObject *params, *views;
  if (!PyArg_ParseTuple(args, "O!O!", &PyTuple_Type, &params, &PyTuple_Type, &views))
    return nullptr;
  const Py_ssize_t n = PyTuple_GET_SIZE(params);
  if (PyTuple_GET_SIZE(views) != n) {
    PyErr_SetString(PyExc_ValueError, "bind_grads: length mismatch");
    return nullptr;
  }
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* t = PyTuple_GET_ITEM(params, i);
    PyObject* v = PyTuple_GET_ITEM(views, i);
    if (!THPVariable_Check(t) || !THPVariable_Check(v)) {
      PyErr_SetString(PyExc_TypeError, "bind_grads: expected tensors");
      return nullptr;
    }
    const at::Tensor& x = THPVariable_Unpack(t);
    const at::Tensor& g = THPVariable_Unpack(v);
    if (g.sizes() != x.sizes() || g.scalar_type() != x.scalar_type() ||
        g.device() != x.device()) {
      PyErr_SetString(PyExc_ValueError, "bind_grads: gradient view does not match its parameter");
      return nullptr;
    }
    x.mutable_grad() = g;
  }
  Py_RETURN_NONE;
}

PyMethodDef kMethods[] = {
    {"grad_state", grad_state, METH_VARARGS, "is every .grad its bucket view / None"},
    {"bind_grads", bind_grads, METH_VARARGS, ".grad = bucket view for every parameter"},
    {"valid_views", valid_views, METH_VARARGS, "arena validity check (see shim.cpp)"},
    {"dict_tags", dict_tags, METH_VARARGS, "PEP 509 version tags of dicts (None: unavailable)"},
    {"valid_tagged", valid_tagged, METH_VARARGS, "tag + data-pointer validity check"},
    {"bump_versions", bump_versions, METH_VARARGS, "autograd version bump of every tensor"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_fa_shim", "feddct_amd host bookkeeping", -1,
                       kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__fa_shim(void) { return PyModule_Create(&kModule); }
