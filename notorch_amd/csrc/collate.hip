// Host-side batched-graph collate (BatchedGraph.from_graphs, notorch/data/models/graph.py:186-223,
// called per batch by MolToGraph.collate, transforms/graph.py:45), SURVEY §8(f) row 3.
//
// One pass over the B per-molecule graphs (caller-owned host buffers):
//   node / edge feature rows copied into the batch (row-major, any element type: rows are bytes);
//   edge_index + cumulative node offset (graph.py:199);
//   rev_index + cumulative NODE offset (rev_mode 0, the reference's graph.py:200 quirk) or
//             + cumulative EDGE offset (rev_mode 1, the fix);
//   batch_node_index / batch_edge_index (graph.py:201-202);
// and, on top of the reference's outputs, the CSR layout the kernels consume:
//   dst_ptr[V+1] / dst_perm[E]: in-edges of every node in ascending edge id (a stable counting sort,
//   O(V + E), the accumulation order of the reference's CPU scatter_add_), mol_ptr[B+1].
// Every local index is validated (src / dst in [0, V_i), rev in [0, E_i)); the first bad one is
// reported and nothing is written past a buffer.  Host memory only, no HIP calls.
#include <string.h>

#include <string>
#include <vector>

#include "common.hpp"

extern "C" int nt_collate_graphs(int64_t B, const void* const* node_feats, const int64_t* n_nodes,
                                 int64_t node_row_bytes, const void* const* edge_feats,
                                 const int64_t* n_edges, int64_t edge_row_bytes,
                                 const int64_t* const* edge_index, const int64_t* const* rev_index,
                                 int rev_mode, void* node_out, void* edge_out,
                                 int64_t* edge_index_out, int64_t* rev_out,
                                 int64_t* batch_node_index, int64_t* batch_edge_index,
                                 int32_t* dst_ptr, int32_t* dst_perm, int32_t* mol_ptr) {
  using namespace nt;
  clear_error();
  NT_REQUIRE(B >= 0 && node_row_bytes >= 0 && edge_row_bytes >= 0, NT_EINVAL, "bad sizes");
  NT_REQUIRE(rev_mode == 0 || rev_mode == 1, NT_EINVAL, "rev_mode must be 0 (nodes) or 1 (edges)");
  NT_REQUIRE(B == 0 || (n_nodes && n_edges && edge_index && rev_index), NT_EINVAL, "NULL pointer");
  int64_t V = 0, E = 0;
  for (int64_t g = 0; g < B; ++g) {
    NT_REQUIRE(n_nodes[g] >= 0 && n_edges[g] >= 0, NT_EINVAL, "negative graph size");
    V += n_nodes[g];
    E += n_edges[g];
  }
  NT_REQUIRE(V < (int64_t(1) << 31) && E < (int64_t(1) << 31), NT_EINVAL,
             "batch too large for the int32 CSR (V, E < 2^31)");
  // edge outputs may be NULL (empty tensors) when the batch has no edge at all
  NT_REQUIRE((E == 0 || (edge_index_out && rev_out && batch_edge_index && dst_perm)) &&
                 (V == 0 || batch_node_index) && dst_ptr && mol_ptr,
             NT_EINVAL, "NULL output pointer");
  NT_REQUIRE(node_row_bytes == 0 || V == 0 || (node_feats && node_out), NT_EINVAL, "NULL node_feats");
  NT_REQUIRE(edge_row_bytes == 0 || E == 0 || (edge_feats && edge_out), NT_EINVAL, "NULL edge_feats");

  // pass 1: copy, offset, validate, count in-degrees
  std::vector<int32_t> deg(V + 1, 0);
  int64_t voff = 0, eoff = 0;
  mol_ptr[0] = 0;
  for (int64_t g = 0; g < B; ++g) {
    const int64_t nv = n_nodes[g], ne = n_edges[g];
    if (node_row_bytes && nv)
      memcpy((char*)node_out + voff * node_row_bytes, node_feats[g], (size_t)(nv * node_row_bytes));
    if (edge_row_bytes && ne)
      memcpy((char*)edge_out + eoff * edge_row_bytes, edge_feats[g], (size_t)(ne * edge_row_bytes));
    const int64_t* ei = edge_index[g];
    const int64_t* rv = rev_index[g];
    NT_REQUIRE(ne == 0 || (ei && rv), NT_EINVAL, "NULL edge_index / rev_index of a graph");
    const int64_t rbase = rev_mode == 0 ? voff : eoff;
    for (int64_t j = 0; j < ne; ++j) {
      const int64_t s = ei[j], d = ei[ne + j], r = rv[j];
      if (s < 0 || s >= nv || d < 0 || d >= nv || r < 0 || r >= ne) {
        set_error("nt_collate_graphs: graph " + std::to_string(g) + " edge " + std::to_string(j) +
                  " has an index out of range (edge_index in [0, " + std::to_string(nv) +
                  "), rev_index in [0, " + std::to_string(ne) + "))");
        return NT_EINVAL;
      }
      edge_index_out[eoff + j] = s + voff;
      edge_index_out[E + eoff + j] = d + voff;
      rev_out[eoff + j] = r + rbase;
      batch_edge_index[eoff + j] = g;
      ++deg[d + voff + 1];
    }
    for (int64_t v = 0; v < nv; ++v) batch_node_index[voff + v] = g;
    voff += nv;
    eoff += ne;
    mol_ptr[g + 1] = (int32_t)voff;
  }
  // pass 2: stable counting sort of the edges by destination
  dst_ptr[0] = 0;
  for (int64_t v = 0; v < V; ++v) dst_ptr[v + 1] = dst_ptr[v] + deg[v + 1];
  std::vector<int32_t> fill(dst_ptr, dst_ptr + V);
  const int64_t* dst = edge_index_out + E;
  for (int64_t e = 0; e < E; ++e) dst_perm[fill[dst[e]]++] = (int32_t)e;
  return NT_OK;
}
