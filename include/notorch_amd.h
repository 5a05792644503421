/*
 * notorch_amd.h — C ABI of the MI355X-native D-MPNN message-passing engine.
 *
 * This is the drop-in boundary for the bond-message D-MPNN forward of davidegraff/notorch
 * (`ChempropBlock` + readout + batched-graph collate).  The reference has no native code of its
 * own: its arithmetic lives in ATen (`index`, `addmm`) and torch_scatter (`scatter_add_`).  Each
 * entry point below replaces the reference call site named in its comment (paths are relative to
 * the reference repository root).
 *
 * Conventions (all entry points):
 *   - plain C types only; device pointers are `void*` / typed pointers into memory the CALLER owns
 *     (PyTorch's caching allocator).  The library never allocates, frees or retains device memory.
 *   - `stream` is a `hipStream_t` passed as `void*` (NULL = the legacy default stream).  Every call
 *     is stream-ordered and asynchronous: no device synchronisation, no host<->device copies, so a
 *     caller may capture the sequence into a hipGraph.
 *   - return value: 0 = NT_OK; nonzero = error, message via nt_last_error() (thread-local).
 *   - row-major feature matrices with leading dimension == h (contiguous rows).
 *   - reference index tensors (edge_index, rev_index, batch_node_index) are int64 exactly as the
 *     reference stores them (graph.py:208-211); engine-built CSR arrays are int32.
 */
#ifndef NOTORCH_AMD_H
#define NOTORCH_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NT_ABI_VERSION 8

#if defined(NT_BUILD)
#define NT_API __attribute__((visibility("default")))
#else
#define NT_API
#endif

enum nt_status { NT_OK = 0, NT_EINVAL = 1, NT_EHIP = 2, NT_EUNSUPPORTED = 3 };

/* element type of feature matrices, weights and bias.  NT_BF16: bf16 storage, fp32 arithmetic, one
 * rounding per stored element (BASELINE config 3); the backward entry points take both. */
enum nt_dtype { NT_F32 = 0, NT_BF16 = 1 };

/* reduce domain of notorch.types.Reduction (types.py:57) with torch_scatter semantics:
 * sum; mean = sum / max(count, 1); max/min of an empty segment = 0. */
enum nt_reduce { NT_SUM = 0, NT_MEAN = 1, NT_MAX = 2, NT_MIN = 3 };

/* element-wise activation applied to messages (ChempropLayer.act, chemprop.py:24,37) */
enum nt_act {
  NT_ACT_IDENTITY = 0,
  NT_ACT_RELU = 1,
  NT_ACT_LEAKY_RELU = 2, /* alpha = negative_slope */
  NT_ACT_ELU = 3,        /* alpha */
  NT_ACT_GELU = 4,       /* erf form */
  NT_ACT_SILU = 5,
  NT_ACT_TANH = 6,
  NT_ACT_SIGMOID = 7
};

/* ABI version of the loaded library (== NT_ABI_VERSION of the header it was built from). */
NT_API int nt_abi_version(void);

/* Message of the last failed call on this thread ("" if none). */
NT_API const char* nt_last_error(void);

/* Which layer-kernel variant the last nt_dmpnn_update / nt_dmpnn_update_fused / nt_dmpnn_dense_matmul
 * call on this thread launched (a static string, e.g. "update_fw_kernel: one 4-wave workgroup per CU,
 * 128-row tiles"; "" before any such call).  For reports and bench labels only. */
NT_API const char* nt_last_kernel(void);

/*
 * GraphEmbedding (notorch/nn/gnn/embed.py:11-36), one sum-mode nn.EmbeddingBag (embed.py:21-22,29):
 *   out[i] = sum_{j < k} table[idx[i * k + j]]          (ascending j, fp32 accumulation)
 * table: num_types x h (dtype); idx: n x k int64 type indices (the featurised node_feats V x 7 or
 * edge_feats E x 2, transforms/graph.py:32-43); out: n x h.  Indices outside [0, num_types) are
 * skipped (the host validates them and raises IndexError as nn.EmbeddingBag would).
 */
NT_API int nt_embed_bag(const void* table, int64_t num_types, const int64_t* idx, int64_t n, int64_t k,
                        int64_t h, int dtype, void* out, void* stream);

/*
 * GraphEmbedding fused into the initial gather (embed.py:29 then
 * chemprop.py:82-83 and layer 0's chemprop.py:37-39), without materialising Xv / Xe:
 *   H0[e] = Xv[src e] + Xe[e],  Xv[s] = sum_j node_table[node_types[s][j]],
 *                               Xe[e] = sum_j edge_table[edge_types[e][j]]
 *   S[v]  = reduce_{e: dst e = v} act(H0[e])   if S != NULL (then seg_ptr / perm = dst CSR)
 * Bit-identical to nt_embed_bag twice followed by nt_dmpnn_init.
 * amax_out (fp32 only, may be NULL): 2 device floats, atomically raised to max|H0| and max|S| (the
 * caller zero-fills them); the fp32 layer kernel scales its fp16 split by them.  ld_out (ABI 7): row
 * pitch in elements of H0 and S (0 = h; > h: fp32 with S, 7 + 2 type columns, as nt_dmpnn_init's).
 * records (ABI 8, may be NULL): nt_embed_edge_records of this graph; with it (fp32, S given, 7 + 2
 * type columns, h % 4 == 0, (num_node_types + num_edge_types + 2) * h * 4 <= 72 KiB) the init runs one
 * wave per node over the records with both tables in LDS (the same bits).
 */
NT_API int nt_dmpnn_init_embed(const void* node_table, int64_t num_node_types,
                               const int64_t* node_types, int64_t kv, const void* edge_table,
                               int64_t num_edge_types, const int64_t* edge_types, int64_t ke,
                               const int64_t* src, const int32_t* seg_ptr, const int32_t* perm,
                               int64_t V, int64_t E, int64_t h, int act, float act_alpha, int reduce,
                               int dtype, void* H0, void* S, float* amax_out, int64_t ld_out,
                               const void* records, void* stream);

/*
 * Type records of a graph for nt_dmpnn_init_embed (ABI 8; no reference counterpart: a layout of the
 * reference's node_feats / edge_feats type columns, transforms/graph.py:32-43): per position p of the
 * dst CSR (perm), 16 B {e = perm[p], node_types[src e][0..6] and edge_types[e][0..1] as bytes}; an
 * out-of-range index is stored as 255 (a zero row).  node_types V x 7, edge_types E x 2 (int64),
 * fewer than 255 types of each kind; records: E x 16 B, 16-B aligned.
 */
NT_API int nt_embed_edge_records(const int64_t* node_types, int64_t num_node_types, const int64_t* edge_types,
                                 int64_t num_edge_types, const int64_t* src, const int32_t* perm, int64_t V,
                                 int64_t E, void* records, void* stream);

/*
 * Host-side collate of B per-molecule graphs (BatchedGraph.from_graphs, notorch/data/models/
 * graph.py:186-223; MolToGraph.collate, transforms/graph.py:45).  HOST memory only, no device call.
 * Inputs per graph g: node_feats[g] (n_nodes[g] rows of node_row_bytes), edge_feats[g] (n_edges[g]
 * rows of edge_row_bytes), edge_index[g] (2 x n_edges[g] int64, row-major), rev_index[g]
 * (n_edges[g] int64), all with graph-local indices.  Outputs (caller-allocated, V = sum n_nodes,
 * E = sum n_edges): the concatenated feature rows, edge_index_out 2 x E (+ node offset, graph.py:199),
 * rev_out E (+ node offset for rev_mode 0 = the reference's graph.py:200, + edge offset for
 * rev_mode 1), batch_node_index V / batch_edge_index E (graph.py:201-202), and the CSR layout:
 * dst_ptr V+1 / dst_perm E (in-edges per node, ascending edge id) and mol_ptr B+1.
 * An out-of-range local index returns NT_EINVAL naming the graph and edge.
 */
NT_API int nt_collate_graphs(int64_t B, const void* const* node_feats, const int64_t* n_nodes,
                             int64_t node_row_bytes, const void* const* edge_feats,
                             const int64_t* n_edges, int64_t edge_row_bytes,
                             const int64_t* const* edge_index, const int64_t* const* rev_index,
                             int rev_mode, void* node_out, void* edge_out, int64_t* edge_index_out,
                             int64_t* rev_out, int64_t* batch_node_index, int64_t* batch_edge_index,
                             int32_t* dst_ptr, int32_t* dst_perm, int32_t* mol_ptr);

/* Number of bytes of device workspace nt_csr_build needs for n indices into nseg segments. */
NT_API size_t nt_csr_workspace_bytes(int64_t n, int64_t nseg);

/*
 * Build a CSR (segment) view of an int64 index vector: seg_ptr[nseg+1], perm[n] such that
 * perm[seg_ptr[s] .. seg_ptr[s+1]) lists every i with idx[i] == s in ASCENDING i (stable), which
 * is the accumulation order of the CPU `scatter_add_` the reference runs.
 * Replaces the implicit segmentation inside torch_scatter.scatter(..., dest, dim_size=V)
 * (notorch/nn/gnn/chemprop.py:39, :86) and scatter_*(..., batch_node_index, dim_size=len(G))
 * (notorch/nn/gnn/agg.py:27, :36, :45).
 * err_flag (device int32, may be NULL): set to 1 if any idx is outside [0, nseg)  (such entries
 * are dropped from the CSR instead of being written out of bounds).
 */
NT_API int nt_csr_build(const int64_t* idx, int64_t n, int64_t nseg, int32_t* seg_ptr, int32_t* perm,
                 void* workspace, size_t workspace_bytes, int32_t* err_flag, void* stream);

/*
 * Initial edge hidden state, optionally fused with the first layer's aggregation:
 *   H0[e] = Xv[src[e]] + Xe[e]                                  (chemprop.py:82-83)
 *   S[v]  = reduce_{e: dst[e]=v} act(H0[e])  if S != NULL       (chemprop.py:37-39, layer 0)
 * src = edge_index[0] (int64, E); (seg_ptr, perm) = nt_csr_build(edge_index[1], E, V).
 * amax_out (fp32 only, may be NULL): 2 device floats, atomically raised to max|H0| and max|S| (S
 * only when S != NULL); the caller zero-fills them.  They are the amax_in of layer 0's
 * nt_dmpnn_update_fused.  ld_out (ABI 7): row pitch in elements of H0 and S (0 = h; > h: fp32 with
 * h % 4 == 0 and ld_out % 4 == 0, the padded rows nt_dmpnn_update_fused's ld_in takes).
 * skip_degree (ABI 7; fp32 with S, h >= 128, 0 = none): nodes with more in-edges are skipped (no H0 rows
 * of their in-edges, no S row): a hub graph's hubs then come from nt_dmpnn_init_chunked over a chunk
 * plan of the hubs alone, so no wave walks a hub's hundreds of in-edges.
 */
NT_API int nt_dmpnn_init(const void* Xv, const void* Xe, const int64_t* src, const int32_t* seg_ptr,
                  const int32_t* perm, int64_t V, int64_t E, int64_t h, int act, float act_alpha,
                  int reduce, int dtype, void* H0, void* S, float* amax_out, int64_t ld_out,
                  int skip_degree, void* stream);

/*
 * max |X| over n fp32 elements, atomically max-ed into *out (device float; non-negative floats
 * order like their bit patterns, so the caller zero-fills it first).  The amax_in of a layer whose
 * inputs did not come from nt_dmpnn_init / nt_dmpnn_update_fused.
 */
NT_API int nt_absmax(const void* X, int64_t n, int dtype, float* out, void* stream);

/*
 * Segmented reduction over CSR segments:
 *   out[s] = reduce_{j in [seg_ptr[s], seg_ptr[s+1])} act(X[perm ? perm[j] : j])
 * Used for the per-layer message aggregation (chemprop.py:37-39), the final node scatter
 * (chemprop.py:86, act = identity) and the Sum/Mean/Max readouts (agg.py:23-47).
 */
NT_API int nt_segment_reduce(const void* X, const int32_t* seg_ptr, const int32_t* perm, int64_t nseg,
                      int64_t h, int reduce, int act, float act_alpha, int dtype, void* out,
                      void* stream);

/*
 * The per-layer message aggregation under the name SURVEY §8(b) gives it (chemprop.py:36-39):
 *   S_out[v] = reduce_{j in [row_ptr[v], row_ptr[v+1])} relu(H[perm[j]])
 * over the dst CSR of nt_csr_build; = nt_segment_reduce(H, row_ptr, perm, V, h, reduce,
 * NT_ACT_RELU, 0, dtype, S_out, stream).  The shipping forward fuses this into nt_dmpnn_init and
 * nt_dmpnn_update_fused; this entry point serves callers that run the layer unfused.
 */
NT_API int nt_dmpnn_aggregate(const void* H, const int32_t* row_ptr, const int32_t* perm, int64_t V,
                              int64_t h, int reduce, int dtype, void* S_out, void* stream);

/*
 * nt_segment_reduce for segments of very different lengths (polymer hubs):
 * the CSR positions are cut into chunks [chunk_pos[k], chunk_pos[k+1]) of bounded length that never
 * straddle a segment; segment s owns chunks [chunk_ptr[s], chunk_ptr[s+1]) (none when empty).
 * Pass 1 reduces every chunk into partial (nchunks x h fp32 workspace), pass 2 combines each
 * segment's partials in chunk order (mean divides by seg_ptr's count).  chunk_seg (int32[nchunks],
 * may be NULL): s when chunk k is segment s's only chunk, else -1 — pass 1 then stores that segment's
 * result directly and pass 2 runs only over the ncomb segments listed in comb_seg (int32[ncomb]: every
 * segment with != 1 chunk); with chunk_seg NULL pass 2 runs over all nseg segments and comb_seg /
 * ncomb are ignored.  (ABI 7)  Same result as
 * nt_segment_reduce up to fp32 reassociation at chunk boundaries; deterministic.  amax_out (fp32,
 * may be NULL; ignored for bf16): one zero-filled device float raised to max|out| (the first layer's
 * split scale on hub graphs).
 */
NT_API int nt_segment_reduce_chunked(const void* X, const int32_t* perm, const int32_t* chunk_pos,
                                     int64_t nchunks, const int32_t* chunk_ptr, const int32_t* chunk_seg,
                                     const int32_t* comb_seg, int64_t ncomb, const int32_t* seg_ptr,
                                     int64_t nseg, int64_t h, int reduce, int act, float act_alpha,
                                     int dtype, float* partial, void* out, float* amax_out, void* stream);

/*
 * nt_dmpnn_init fused with layer 0's aggregation on hub graphs (fp32): the chunked reduction above with
 * the rows computed in pass 1 instead of read, H0[e] = Xv[src[e]] + Xe[e] (chemprop.py:82-83) stored
 * as it goes, then S[v] = reduce act(H0) over v's chunks (chemprop.py:37-39, layer 0), so H0 is
 * written once and never re-read.  (perm, chunk_pos, chunk_ptr, chunk_seg, comb_seg, ncomb, seg_ptr) as
 * nt_segment_reduce_chunked
 * on the dst CSR; H0 E x h, S V x h.  Same H0 as nt_dmpnn_init (bit-identical), same S as
 * nt_segment_reduce_chunked of that H0.  amax_out (may be NULL): 2 zero-filled device floats raised to
 * max|H0|, max|S|.  ld_out (ABI 7): row pitch in elements of H0 and S (0 = h; >= h, a multiple of 4;
 * the partial rows stay dense).  chunk_ids (ABI 7, may be NULL): pass 1 runs only these nids chunks of
 * the plan (a hub graph's hub chunks, after nt_dmpnn_init with skip_degree wrote the other nodes).
 * Pass 2 still combines every segment in comb_seg, so chunk_ids must list EVERY chunk of every
 * multi-chunk segment: with skip_degree <= the plan's chunk rows (kernels.CHUNK_ROWS = 32), each node
 * nt_dmpnn_init skipped has all its chunks listed and each node it wrote is a single chunk.
 */
NT_API int nt_dmpnn_init_chunked(const void* Xv, const void* Xe, const int64_t* src, const int32_t* perm,
                                 const int32_t* chunk_pos, int64_t nchunks, const int32_t* chunk_ptr,
                                 const int32_t* chunk_seg, const int32_t* comb_seg, int64_t ncomb,
                                 const int32_t* seg_ptr, int64_t V, int64_t E, int64_t h, int act,
                                 float act_alpha, int reduce, int dtype, float* partial, void* H0, void* S,
                                 float* amax_out, int64_t ld_out, const int32_t* chunk_ids, int64_t nids,
                                 void* stream);

/* Bytes of the packed weight image for one h x h layer (see nt_dmpnn_pack_weight). */
NT_API size_t nt_dmpnn_packed_weight_bytes(int64_t h, int dtype);

/*
 * Repack `nlayers` nn.Linear weights W_l [h_out = h][h_in = h] (row-major, chemprop.py:26) into
 * the MFMA fragment image nt_dmpnn_update consumes.  W points at nlayers contiguous h*h matrices
 * (or use nlayers = 1 per layer); Wp at nlayers * nt_dmpnn_packed_weight_bytes(h) bytes.
 */
NT_API int nt_dmpnn_pack_weight(const void* W, int64_t nlayers, int64_t h, int dtype, void* Wp,
                         void* stream);

/*
 * fp32 only: the part of nt_dmpnn_pack_weight's image that the fp32 layer kernel reads (its
 * two-part fp16 image and scale), at the same offsets; the other parts of Wp are left untouched.
 * Enough for nt_dmpnn_update_fused and nt_dmpnn_dense_matmul (the backward packs W^T this way
 * every step).  Replaces the same call sites as nt_dmpnn_pack_weight (chemprop.py:26,41).
 */
NT_API int nt_dmpnn_pack_weight_fk(const void* W, int64_t nlayers, int64_t h, void* Wp, void* stream);

/*
 * nt_dmpnn_pack_weight_fk for nlayers (<= 16) separate h x h weights in one launch pair: W, Wp (and
 * WpT) are HOST arrays of nlayers device pointers; WpT may be NULL, else WpT[l] receives the fk
 * image of W[l]^T (the backward's dA = G W, chemprop.py:41 under autograd) read from W[l] directly.
 * Same bytes as nt_dmpnn_pack_weight_fk of W[l] and of W[l].t().contiguous().
 */
NT_API int nt_dmpnn_pack_weights_fk(const void* const* W, int64_t nlayers, int64_t h, void* const* Wp,
                                    void* const* WpT, void* stream);

/*
 * One fused D-MPNN layer (ChempropLayer.forward, chemprop.py:28-43, wrapped by Residual,
 * residual.py:27-28), for every directed edge e:
 *   H_out[e] = (residual ? H[e] : 0) + W (S[src[e]] - act(H[rev[e]])) + b
 * H, S: E x h and V x h; src = edge_index[0], rev = rev_index (int64, arbitrary gather index);
 * Wp = nt_dmpnn_pack_weight image of W; b may be NULL (bias=False).  H_out must not alias H.
 * fp32 with h % 4 == 0 runs the fp16x3 layer kernel: H, S, H_out and b must then be 16-byte aligned
 * (NT_EINVAL otherwise), and amax_ws must point at 2 floats of caller-owned device memory that the
 * call overwrites on `stream` with (max|H|, max|S|) before the layer reads them (the split scales;
 * stream-ordered: reuse it only for work ordered after this call).  amax_ws may be NULL for bf16 and
 * for h % 4 != 0 (the exact fp32 tile kernel).  (ABI 6: the library holds no device scratch.)
 */
NT_API int nt_dmpnn_update(const void* H, const void* S, const int64_t* src, const int64_t* rev,
                    const void* Wp, const void* b, int64_t V, int64_t E, int64_t h, int residual,
                    int act, float act_alpha, int dtype, float* amax_ws, void* H_out, void* stream);

/*
 * Tile plan for nt_dmpnn_update_fused: cuts the dst-sorted edge order (positions of the
 * nt_csr_build(edge_index[1]) permutation) at node boundaries, so every node's in-edges fall in one
 * tile.  Tile k starts at dst_ptr[first v with dst_ptr[v] >= k stride]; tile_ptr[ntiles] = E; a
 * tile then holds at most stride + max_in_degree - 1 positions.  dst_sorted[p] = the node whose
 * in-edge sits at position p.
 * nt_dmpnn_tile_stride(E, max_in_degree, rows, ncu): the stride for tiles of at most `rows`
 * positions (rows = nt_dmpnn_fused_tile_rows), balanced so that the tile count is a whole number of
 * rounds of ncu tiles (ncu <= 0: the largest stride); 0 when max_in_degree > rows.
 * ntiles must equal nt_dmpnn_tile_count(E, stride).  Graphs whose max in-degree exceeds 32 take the
 * unfused path (nt_dmpnn_update_fused without a plan + nt_segment_reduce).
 * Replaces the per-layer segmentation implied by scatter(..., dest) (chemprop.py:39, :86).
 */
NT_API int64_t nt_dmpnn_tile_stride(int64_t E, int max_in_degree, int rows, int ncu);
NT_API int64_t nt_dmpnn_tile_count(int64_t E, int64_t stride);
NT_API int nt_dmpnn_tile_plan(const int32_t* dst_ptr, int64_t V, int64_t E, int64_t stride,
                              int32_t* tile_ptr, int64_t ntiles, int32_t* dst_sorted, void* stream);

/*
 * nt_dmpnn_tile_plan for graphs with hub nodes (in-degree > hub_degree, e.g. polymer hubs,
 * BASELINE config 5): the same plan, except that a target k * stride inside a hub's in-edges cuts
 * the tile there instead of rounding up to the next node.  stride = nt_dmpnn_tile_stride with
 * max_in_degree = the largest in-degree among the non-hub nodes (<= hub_degree <= 32).  The fused
 * layer then takes the row table marked by nt_dmpnn_mark_hub_rows and leaves the hubs' S_out rows
 * to nt_dmpnn_hub_aggregate.  Replaces the segmentation of scatter(..., dest) (chemprop.py:39, :86)
 * for the hub nodes.  nt_dmpnn_tile_plan = this with hub_degree = INT32_MAX.
 */
NT_API int nt_dmpnn_tile_plan_hubs(const int32_t* dst_ptr, int64_t V, int64_t E, int64_t stride,
                                   int hub_degree, int32_t* tile_ptr, int64_t ntiles, int32_t* dst_sorted,
                                   void* stream);

/*
 * Marks the hub rows of a row table (nt_dmpnn_row_table) in place: every dst-sorted position whose
 * node has more than hub_degree in-edges (dst_ptr: the dst CSR) becomes a segment start without a
 * segment end, so nt_dmpnn_update_fused stores those rows' H_out but none of the hub's S_out.
 */
NT_API int nt_dmpnn_mark_hub_rows(void* row_table, int64_t E, const int32_t* dst_ptr, int64_t V,
                                  int hub_degree, void* stream);

/*
 * The hubs' share of a fused layer's aggregation (chemprop.py:37-39, :86; torch_scatter semantics):
 *   out[v] = reduce_{p in [seg_ptr[v], seg_ptr[v+1])} act(X[perm[p]])   for v in hubs[0 .. nhub)
 * (rows of other nodes untouched).  amax_out (may be NULL): one device float raised to max|out[v]|
 * (the fused layer's max|S_out| slot).  fp32, h % 4 == 0, 16-byte aligned X / out; deterministic
 * (16 contiguous row ranges per hub, combined in order).  ld (ABI 7): row pitch in elements of X and
 * out (0 = h; >= h, a multiple of 4).
 */
/*
 * The fused layer's hub partials combined (ABI 7): with S_part given to nt_dmpnn_update_fused and a
 * row table whose hub rows are sub-runs (entries -((slot << 2) | start | end << 1) - 1: runs of one
 * hub's consecutive in-edges within a tile, at most max_in_degree rows each), the layer stores each
 * sub-run's reduce of agg_act(H_out) as partial row `slot` (fp32, h wide, dense); then for v in hubs
 *   out[v] = reduce_{k in [slot_ptr[v], slot_ptr[v+1])} partial[k]   (mean: / in-degree from seg_ptr)
 * slot_ptr (int32[V+1]): slots before node v's rows.  Combined as nt_segment_reduce_chunked's pass 2
 * (32 consecutive sub-ranges in order; deterministic).  amax_out (may be NULL): one device float
 * raised to max|out[hubs]|.  fp32, h % 4 == 0; ld = row pitch in elements of out (0 = h).
 */
NT_API int nt_dmpnn_hub_combine(const void* partial, const int32_t* hubs, const int32_t* slot_ptr, int64_t nhub,
                                const int32_t* seg_ptr, int64_t V, int64_t h, int reduce, int dtype,
                                float* amax_out, void* out, int64_t ld, void* stream);

NT_API int nt_dmpnn_hub_aggregate(const void* X, const int32_t* perm, const int32_t* seg_ptr,
                                  const int32_t* hubs, int64_t nhub, int64_t h, int reduce, int act,
                                  float act_alpha, int dtype, float* amax_out, void* out, int64_t ld,
                                  void* stream);

/*
 * Row capacity of one nt_dmpnn_update_fused tile for a layer of hidden size h, activation act and
 * aggregation (reduce, agg_act): the plan passed with that layer must have tiles of at most this
 * many rows.  fp32: 128 for h <= 384 with act = relu, reduce = sum and agg_act in {relu,
 * identity}, else 64; bf16: 64.
 */
NT_API int nt_dmpnn_fused_tile_rows(int64_t h, int dtype, int act, int reduce, int agg_act);

/*
 * One D-MPNN layer fused with the aggregation that consumes it (chemprop.py:36-43 of layer l,
 * residual.py:27-28, then chemprop.py:37-39 of layer l+1 or, with agg_act = NT_ACT_IDENTITY, the
 * final node scatter of chemprop.py:86):
 *   H_out[e] = (residual ? H[e] : 0) + W (S[src[e]] - act(H[rev[e]])) + b
 *   S_out[v] = reduce_{e: dst[e]=v} agg_act(H_out[e])      (ascending e; empty segment -> 0)
 * (tile_ptr, ntiles, dst_sorted) = nt_dmpnn_tile_plan with tiles of at most tile_rows <=
 * nt_dmpnn_fused_tile_rows(h, dtype, act, reduce, agg_act) rows; max_in_degree >= the graph's largest
 * in-degree (<= 32); perm = the dst CSR permutation (bf16); row_table = nt_dmpnn_row_table (fp32).
 * Nodes without in-edges are not written (the caller zero-fills S_out).  With tile_ptr = NULL (and perm, dst_sorted, S_out = NULL) only H_out
 * is computed.
 * fp32 (h % 4 == 0, any h): two-part fp16 split on fp16 MFMA (fp32 accuracy); amax_in = 2 device
 * floats >= max|H|, max|S| (from nt_dmpnn_init / the previous layer's amax_out / nt_absmax);
 * amax_out (may be NULL) = 2 zero-filled device floats raised to max|H_out|, max|S_out|.
 * bf16 (h % 8 == 0, h <= 512): bf16 MFMA, tile_rows <= 64, amax ignored.
 * 16-byte aligned feature pointers; S_out must not alias S.
 * S_part (ABI 7, fp32, may be NULL): the hub partial rows (nt_dmpnn_hub_combine) when the row table
 * marks hub sub-runs.
 * ld_in / ld_out (ABI 7): row pitch in elements of H and S / of H_out and S_out (0 = h; fp32: >= h and
 * a multiple of 4, bf16: h).  Rows padded to a 32-byte multiple (h = 300 -> 304) keep every row's
 * pieces on whole 32-B sectors: the intermediate layers of a forward run on padded rows.
 */
NT_API int nt_dmpnn_update_fused(const void* H, const void* S, const int64_t* src, const int64_t* rev,
                                 const void* Wp, const void* b, int64_t V, int64_t E, int64_t h,
                                 int residual, int act, float act_alpha, const int32_t* tile_ptr,
                                 int64_t ntiles, int tile_rows, int max_in_degree, const int32_t* perm,
                                 const int32_t* dst_sorted, const void* row_table, int reduce,
                                 int agg_act, float agg_alpha, int dtype, const float* amax_in,
                                 float* amax_out, void* H_out, void* S_out, void* S_part, int64_t ld_in,
                                 int64_t ld_out, void* stream);

/*
 * Row table of a fused plan for the fp32 layer kernel: one int32 x 4 entry per dst-sorted position p
 *   { e = perm[p], src[e] (-1 if outside [0, V)), rev[e] (-1 if outside [0, E)),
 *     (dst_sorted[p] << 2) | (first in-edge of its node) | (last in-edge of its node) << 1 }
 * so the kernel reaches a tile's rows in one dependent load.  Depends only on the graph (cache it
 * with the plan).  V < 2^29, E < 2^31; out: E x 16 bytes, 16-byte aligned.
 */
NT_API int nt_dmpnn_row_table(const int32_t* perm, const int32_t* dst_sorted, const int64_t* src,
                              const int64_t* rev, int64_t V, int64_t E, void* out, void* stream);

/*
 * Attention readout scores (notorch/nn/gnn/agg.py:50-86), one per node row X[v] (n x h):
 *   Gated        (a != NULL, Q == NULL): s[v] = X[v] . a + (a_bias ? *a_bias : 0)   (agg.py:53,59)
 *   SDPAttention (Q != NULL, a == NULL): s[v] = (Q[node_seg[v]] . X[v]) / sqrt_key   (agg.py:79-82)
 * a: h (the nn.Linear(d, 1) weight row), Q: nseg x h, node_seg = batch_node_index (int64);
 * scores: n fp32.
 */
NT_API int nt_node_scores(const void* X, int64_t n, int64_t h, const void* a, const void* a_bias,
                          const void* Q, const int64_t* node_seg, float sqrt_key, int dtype,
                          float* scores, void* stream);

/*
 * Softmax-weighted segment sum (agg.py:60-61, :83-84: scatter_softmax then scatter_sum):
 *   alpha[v] = exp(s[v] - max_g s) / sum_{u in g} exp(s[u] - max_g s)
 *   out[g]   = sum_{v in g} alpha[v] X[v]          (ascending v; empty segment -> 0)
 * (seg_ptr, perm) = nt_csr_build(batch_node_index, n, nseg); perm may be NULL if sorted.
 */
NT_API int nt_softmax_pool(const void* X, const float* scores, const int32_t* seg_ptr,
                           const int32_t* perm, int64_t nseg, int64_t h, int dtype, void* out,
                           void* stream);

/*
 * Backward of nt_node_scores + nt_softmax_pool (the Gated / SDPAttention readouts trained through
 * lightning_models/model.py:224-241; reference: ATen autograd of agg.py:50-86).  For dout (nseg x h):
 *   dalpha[v] = <dout[g], X[v]>,  c_g = <dout[g], out[g]>,  ds[v] = alpha[v] (dalpha[v] - c_g)
 *   dX[v]     = alpha[v] dout[g] + ds[v] key[v]   (key = a: Gated; Q[g] / sqrt_key: SDPA)
 *   P[g]      = sum_{v in g} ds[v] X[v]           (ascending v, fp32; Gated: da = sum_g P[g],
 *                                                  db = sum_v ds[v]; SDPA: dQ = P / sqrt_key)
 * alpha is recomputed exactly as nt_softmax_pool computes it.  X, out, dout, a / Q, dX: dtype;
 * scores, ds (n), P (nseg x h), stats (3 nseg workspace): fp32.  node_seg = batch_node_index.
 */
NT_API int nt_softmax_pool_backward(const void* X, const float* scores, const int32_t* seg_ptr,
                                    const int32_t* perm, const int64_t* node_seg, int64_t nseg, int64_t n,
                                    int64_t h, const void* out, const void* dout, const void* a,
                                    const void* Q, float sqrt_key, int dtype, float* stats, void* dX,
                                    float* ds, float* P, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Backward (training through ChempropBlock, lightning_models/model.py:224-241).  The reference's
 * backward is ATen autograd of chemprop.py:28-43,81-88 (index_backward = index_add, scatter_add
 * backward = gather, addmm backward = two mm).  These replace the gather/scatter/element-wise parts;
 * the two dense products per layer (dA = G W, dW = G^T A) are library GEMMs on the same stream.
 * --------------------------------------------------------------------------------------------- */

/*
 * Layer message, recomputed for the weight gradient (chemprop.py:40):
 *   A[e] = S[src[e]] - act(H[rev[e]])
 */
NT_API int nt_dmpnn_message(const void* H, const void* S, const int64_t* src, const int64_t* rev,
                            int64_t V, int64_t E, int64_t h, int act, float act_alpha, int dtype,
                            void* A_out, void* stream);

/*
 * Gradient of one layer's input hidden state (backward of chemprop.py:37-40 and residual.py:28):
 *   G_out[e] = (residual ? G[e] : 0)
 *            + act'(H[e]) * (dS[dst[e]] / c(dst[e]) - sum_{j in [rev_ptr[e], rev_ptr[e+1])} dA[rev_perm[j]])
 * G = dL/dH_{l+1}; H = H_l; dA = G W; dS = nt_segment_reduce(dA, src CSR, sum);
 * (rev_ptr, rev_perm) = nt_csr_build(rev_index, E, E); c(v) = max(in-degree, 1) for
 * reduce = NT_MEAN (dst_ptr required), 1 for NT_SUM.  max/min are not covered (NT_EUNSUPPORTED).
 * amax_out (fp32, may be NULL; ignored for bf16): one zero-filled device float raised to max|G_out|,
 * the split scale of the backward's fp16-split kernels (nt_dmpnn_weight_grad_fk, dense dA).
 */
NT_API int nt_dmpnn_edge_backward(const void* G, const void* H, const void* dA, const void* dS,
                                  const int64_t* dst, const int32_t* rev_ptr, const int32_t* rev_perm,
                                  const int32_t* dst_ptr, int64_t V, int64_t E, int64_t h,
                                  int residual, int act, float act_alpha, int reduce, int dtype,
                                  void* G_out, float* amax_out, void* stream);

/*
 * Row gather with optional base and mean scaling (backward of a sum/mean scatter):
 *   out[i] = (base ? base[i] : 0) + X[idx[i]] / (seg_ptr ? max(seg_ptr[idx+1] - seg_ptr[idx], 1) : 1)
 * Used for dL/dH_d += dnode[dst] (chemprop.py:86) and the Sum/Mean readout backward
 * (agg.py:23-38, idx = batch_node_index, seg_ptr = molecule CSR for mean).
 * amax_out: as nt_dmpnn_edge_backward (max|out|).
 */
NT_API int nt_gather_rows(const void* base, const void* X, const int64_t* idx, const int32_t* seg_ptr,
                          int64_t n, int64_t nseg, int64_t h, int dtype, void* out, float* amax_out,
                          void* stream);

/* Dropout of the layer update fused with its residual add: replaces `nn.Dropout(p)` inside
 * ChempropLayer.update (notorch/nn/gnn/chemprop.py:26, applied at :42) followed by
 * Residual's `inputs[0] + module(*inputs)` (notorch/nn/residual.py:28), training mode.
 *   out[i] = (base ? base[i] : 0) + keep(seed, offset + i) * Y[i] / (1 - p),   i < n
 * keep() is a counter-based hash (no mask is stored); P(keep) = 1 - p; p = 1 drops every element.
 * The backward is the same call on the incoming gradient with base = NULL and the same
 * (seed, offset).  out may alias base or Y. */
NT_API int nt_dropout_residual(const void* base, const void* Y, int64_t n, float p, uint64_t seed,
                               uint64_t offset, int dtype, void* out, void* stream);

/* Backward of the max / min scatters (torch_scatter scatter_max / scatter_min at chemprop.py:39,86
 * and agg.py:45; trained through lightning_models/model.py:224-241): the gradient of an output
 * element goes to its arg, the FIRST row of the segment (ascending CSR order) holding the extreme.
 *   nt_segment_arg:             arg[v][c] = that row of act(X) over segment v (seg_ptr / perm as
 *                               nt_segment_reduce), -1 for an empty segment; reduce = NT_MAX | NT_MIN
 *   nt_dmpnn_edge_backward_arg: nt_dmpnn_edge_backward with the dS term masked by arg (reduce of the
 *                               layer's aggregation = max | min): (arg[dst e][c] == e ? dS[dst e][c] : 0)
 *   nt_gather_rows_arg:         out[i] = (base ? base[i] : 0) + (arg[idx i] == i ? X[idx i] : 0)
 * fp32 or bf16 storage (bf16: values widened exactly, compared / masked in fp32, one rounding at the
 * store; amax_out must be NULL); amax_out (fp32) as nt_dmpnn_edge_backward. */
NT_API int nt_segment_arg(const void* X, const int32_t* seg_ptr, const int32_t* perm, int64_t nseg,
                          int64_t h, int reduce, int act, float act_alpha, int dtype, int32_t* arg,
                          void* stream);
NT_API int nt_dmpnn_edge_backward_arg(const void* G, const void* H, const void* dA, const void* dS,
                                      const int32_t* arg, const int64_t* dst, const int32_t* rev_ptr,
                                      const int32_t* rev_perm, int64_t V, int64_t E, int64_t h,
                                      int residual, int act, float act_alpha, int dtype, void* G_out,
                                      float* amax_out, void* stream);
NT_API int nt_gather_rows_arg(const void* base, const void* X, const int64_t* idx, const int32_t* arg,
                              int64_t n, int64_t h, int dtype, void* out, float* amax_out, void* stream);

/* Dense layer GEMM, the backward's dA = G W of nn.Linear (chemprop.py:26,41), trained through
 * lightning_models/model.py:224-241 (the reference runs it as ATen addmm's autograd):
 *   out[i] = X[i] W^T,  i < M,   Wp = nt_dmpnn_pack_weight image of W (h x h; pass the image of W^T
 * for dA = G W).  fp32 (h % 4 == 0, 16-byte aligned, out != X): the fp16x3 layer kernel without
 * gathers; amax_in = 2 device floats whose [1] >= max|X| (e.g. written by the kernel that produced
 * X), or NULL: then amax_ws (2 floats of caller-owned device memory, required) receives
 * (0, max|X|) on `stream` first.  bf16 (h <= 512): the bf16 layer kernel, amax_in / amax_ws unused. */
NT_API int nt_dmpnn_dense_matmul(const void* X, int64_t M, int64_t h, const void* Wp, int dtype,
                                 const float* amax_in, float* amax_ws, void* out, void* stream);

/* Weight and bias gradient of one layer (backward of nn.Linear at chemprop.py:26,41, trained through
 * lightning_models/model.py:224-241; the reference runs it as ATen addmm's autograd), with the
 * layer message formed on the fly (never written):
 *   A[e] = S[src[e]] - act(H[rev[e]])   (chemprop.py:40; src = rev = NULL: A[e] = S[e], H unused)
 *   dW = G^T A  (h x h),   db = sum_e G[e]  (db_out may be NULL)
 * Split-K bf16x6 MFMA kernel (fp32-accurate), deterministic (partials reduced in fixed order).
 * workspace: device buffer of at least nt_dmpnn_weight_grad_workspace(E, h) bytes.  fp32 only. */
NT_API int64_t nt_dmpnn_weight_grad_workspace(int64_t E, int64_t h);
NT_API int nt_dmpnn_weight_grad(const void* G, const void* H, const void* S, const int64_t* src,
                                const int64_t* rev, int64_t V, int64_t E, int64_t h, int act,
                                float act_alpha, int dtype, void* workspace, int64_t workspace_bytes,
                                void* dW_out, void* db_out, void* stream);

/* nt_dmpnn_weight_grad on the fp32 layer kernel's numerics (h <= 320, src and rev given): G and A
 * scaled by powers of two from device bounds and split into two fp16 parts, three fp16 MFMA products
 * per tile (fp32-accurate: the dropped term and the split roundings are ~2^-22 relative); half the
 * MFMA work of the bf16x6 kernel.  amax_G: one device float >= max|G|; amax_HS: two device floats
 * >= max|H|, max|S| (the forward's amax chain row of this layer).  Same workspace and outputs. */
NT_API int nt_dmpnn_weight_grad_fk(const void* G, const void* H, const void* S, const int64_t* src,
                                   const int64_t* rev, int64_t V, int64_t E, int64_t h, int act,
                                   float act_alpha, const float* amax_G, const float* amax_HS, int dtype,
                                   void* workspace, int64_t workspace_bytes, void* dW_out, void* db_out,
                                   void* stream);

#ifdef __cplusplus
}
#endif

#endif /* NOTORCH_AMD_H */
