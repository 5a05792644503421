// Host-side helper of the native collate (CPython extension `notorch_amd.lib._collate_py`).
//
// BatchedGraph.from_graphs (reference notorch/data/models/graph.py:186-223) walks a list of
// per-molecule Graphs.  The copies, offsets and CSR are one C++ pass (nt_collate_graphs); what bounded
// the collate was the per-graph Python work that fed it: four attribute reads, contiguity / dtype /
// row-shape checks, sizes and data pointers per graph, ~18 interpreted passes over 4096 graphs
// (~6 ms of a ~8 ms collate at config 2).  graph_arrays() does that walk in one C++ loop over the
// tensors' ATen handles.
//
//   graph_arrays(graphs) -> (status, n_nodes[B] int64, n_edges[B] int64, ptrs[4, B] int64, V, E)
//
// status 0: every graph's node_feats / edge_feats / edge_index / rev_index is a contiguous CPU tensor,
//           the indices int64; ptrs rows = data pointers of node_feats, edge_feats, edge_index,
//           rev_index.  The tensors stay owned by the graphs (the caller keeps the list alive).
// status 1: take the Python path (a tensor is not on the CPU, not contiguous, not int64 where an index
//           must be, 0-dimensional, or an attribute is not a tensor); nothing else is returned.
// status 2 / 3: node_feats / edge_feats of the graphs differ in dtype or row shape.
// status 4: edge_index / rev_index sizes do not match edge_feats.
// The caller raises the reference's errors for 2-4 (graph.py _native_collate).
#include <Python.h>

#include <stdint.h>

#include <ATen/ops/empty.h>
#include <torch/csrc/autograd/python_variable.h>

namespace {

PyObject* g_names[4] = {nullptr, nullptr, nullptr, nullptr};

bool same_rows(const at::Tensor& a, const at::Tensor& b) {
  if (a.scalar_type() != b.scalar_type() || a.dim() != b.dim()) return false;
  for (int64_t d = 1; d < a.dim(); ++d)
    if (a.size(d) != b.size(d)) return false;
  return true;
}

PyObject* status_only(int s) { return Py_BuildValue("(i)", s); }

PyObject* graph_arrays(PyObject*, PyObject* arg) {
  PyObject* seq = PySequence_Fast(arg, "graph_arrays expects a sequence of graphs");
  if (!seq) return nullptr;
  const Py_ssize_t B = PySequence_Fast_GET_SIZE(seq);
  PyObject** items = PySequence_Fast_ITEMS(seq);
  if (B == 0) {
    Py_DECREF(seq);
    return status_only(1);
  }
  at::Tensor nn = at::empty({(int64_t)B}, at::kLong), ne = at::empty({(int64_t)B}, at::kLong);
  at::Tensor ptrs = at::empty({4, (int64_t)B}, at::kLong);
  int64_t* pn = nn.data_ptr<int64_t>();
  int64_t* pe = ne.data_ptr<int64_t>();
  int64_t* pp = ptrs.data_ptr<int64_t>();
  int64_t V = 0, E = 0;
  int status = 0;
  at::Tensor first[2];
  for (Py_ssize_t i = 0; i < B && status == 0; ++i) {
    PyObject* obj[4];
    int got = 0;
    // dataclass graphs keep their fields in the instance dict: four dict lookups on interned names
    // (attribute lookup first walks the type's MRO for descriptors); anything else, or a miss, takes
    // the generic attribute lookup
    PyObject** dictp = _PyObject_GetDictPtr(items[i]);
    PyObject* dict = dictp ? *dictp : nullptr;
    for (; got < 4; ++got) {
      PyObject* v = dict ? PyDict_GetItemWithError(dict, g_names[got]) : nullptr;
      if (v) {
        Py_INCREF(v);
        obj[got] = v;
        continue;
      }
      if (PyErr_Occurred()) PyErr_Clear();
      obj[got] = PyObject_GetAttr(items[i], g_names[got]);
      if (!obj[got]) break;
    }
    if (got < 4) {  // a missing attribute: the Python path raises the reference's AttributeError
      PyErr_Clear();
      for (int k = 0; k < got; ++k) Py_DECREF(obj[k]);
      status = 1;
      break;
    }
    for (int k = 0; k < 4 && status == 0; ++k) {
      if (!THPVariable_Check(obj[k])) {
        status = 1;
        break;
      }
      const at::Tensor& t = THPVariable_Unpack(obj[k]);
      if (!t.device().is_cpu() || !t.is_contiguous() || t.dim() == 0 || (k >= 2 && t.scalar_type() != at::kLong)) {
        status = 1;
        break;
      }
      pp[k * B + i] = (int64_t)(intptr_t)t.data_ptr();
    }
    if (status == 0) {
      const at::Tensor& nf = THPVariable_Unpack(obj[0]);
      const at::Tensor& ef = THPVariable_Unpack(obj[1]);
      if (i == 0) {
        first[0] = nf;
        first[1] = ef;
      } else if (!same_rows(nf, first[0])) {
        status = 2;
      } else if (!same_rows(ef, first[1])) {
        status = 3;
      }
      if (status == 0) {
        const int64_t n = nf.size(0), m = ef.size(0);
        if (THPVariable_Unpack(obj[2]).numel() != 2 * m || THPVariable_Unpack(obj[3]).numel() != m) status = 4;
        pn[i] = n;
        pe[i] = m;
        V += n;
        E += m;
      }
    }
    for (int k = 0; k < 4; ++k) Py_DECREF(obj[k]);
  }
  Py_DECREF(seq);
  if (status != 0) return status_only(status);
  PyObject* r = PyTuple_New(6);
  PyTuple_SET_ITEM(r, 0, PyLong_FromLong(0));
  PyTuple_SET_ITEM(r, 1, THPVariable_Wrap(nn));
  PyTuple_SET_ITEM(r, 2, THPVariable_Wrap(ne));
  PyTuple_SET_ITEM(r, 3, THPVariable_Wrap(ptrs));
  PyTuple_SET_ITEM(r, 4, PyLong_FromLongLong(V));
  PyTuple_SET_ITEM(r, 5, PyLong_FromLongLong(E));
  return r;
}

// The layout's dst-sorted node ids and degree range (graph.py host_stats) in one pass instead of
// numpy's diff / repeat / max / min chain.
bool cpu_contig(PyObject* arg, at::ScalarType st, const at::Tensor** out) {
  if (!THPVariable_Check(arg)) return false;
  const at::Tensor& t = THPVariable_Unpack(arg);
  if (!t.device().is_cpu() || !t.is_contiguous() || t.scalar_type() != st) return false;
  *out = &t;
  return true;
}

// segment_ids(seg_ptr: int32[n + 1] CPU) -> (ids int32[seg_ptr[n]], max count, min count): ids[p] = the
// segment holding position p (np.repeat(arange(n), diff(seg_ptr))); None for a non-monotone pointer
PyObject* segment_ids(PyObject*, PyObject* arg) {
  const at::Tensor* t;
  if (!cpu_contig(arg, at::kInt, &t) || t->dim() != 1 || t->numel() < 1) {
    PyErr_SetString(PyExc_TypeError, "segment_ids expects a contiguous int32 CPU tensor of n + 1 >= 1 offsets");
    return nullptr;
  }
  const int32_t* sp = t->data_ptr<int32_t>();
  const int64_t n = t->numel() - 1;
  if (sp[0] != 0) Py_RETURN_NONE;
  for (int64_t v = 0; v < n; ++v)
    if (sp[v + 1] < sp[v]) Py_RETURN_NONE;
  at::Tensor ids = at::empty({(int64_t)sp[n]}, at::kInt);
  int32_t* __restrict__ o = ids.data_ptr<int32_t>();
  int64_t mx = 0, mn = n > 0 ? INT64_MAX : 0;
  int32_t b = sp[0];
  for (int64_t v = 0; v < n; ++v) {
    const int32_t e = sp[v + 1];
    const int64_t c = e - b;
    mx = c > mx ? c : mx;
    mn = c < mn ? c : mn;
    for (int32_t p = b; p < e; ++p) o[p] = (int32_t)v;
    b = e;
  }
  return Py_BuildValue("(NLL)", THPVariable_Wrap(ids), (long long)mx, (long long)mn);
}

PyMethodDef kMethods[] = {
    {"graph_arrays", graph_arrays, METH_O,
     "graph_arrays(graphs) -> (status, n_nodes, n_edges, ptrs, V, E): the native collate's per-graph inputs"},
    {"segment_ids", segment_ids, METH_O,
     "segment_ids(seg_ptr int32) -> (ids int32, max count, min count), or None if seg_ptr is not monotone"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_collate_py", "host helper of the native collate", -1, kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__collate_py() {
  const char* names[4] = {"node_feats", "edge_feats", "edge_index", "rev_index"};
  for (int k = 0; k < 4; ++k) {
    g_names[k] = PyUnicode_InternFromString(names[k]);
    if (!g_names[k]) return nullptr;
  }
  return PyModule_Create(&kModule);
}
