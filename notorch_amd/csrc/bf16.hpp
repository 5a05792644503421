// Internal interface of the bf16 storage path (bf16.hip): feature rows, weights and bias stored as
// bf16, every sum / product accumulated in fp32 and rounded to bf16 once per stored element.
// Entry points in segment.hip / update_f32.hip forward here when dtype == NT_BF16.
#pragma once

#include "common.hpp"

namespace nt {

int launch_segment_reduce_bf16(const void* X, const int32_t* seg_ptr, const int32_t* perm,
                               int64_t nseg, int64_t h, int reduce, int act, float alpha, void* out,
                               hipStream_t stream);

int launch_init_bf16(const void* Xv, const void* Xe, const int64_t* src, const int32_t* seg_ptr,
                     const int32_t* perm, int64_t V, int64_t E, int64_t h, int act, float alpha,
                     int reduce, void* H0, void* S, hipStream_t stream);

// packed bf16 weight image: [K/32][ceil(h/16)][64 lanes] x 16 B (one MFMA B fragment per lane)
size_t bf16_image_bytes(int64_t h);
int pack_weight_bf16(const void* W, int64_t nlayers, int64_t h, int64_t layer_stride_bytes, void* Wp,
                     hipStream_t stream);

int launch_update_bf16(const void* H, const void* S, const int64_t* src, const int64_t* rev,
                       const void* Wp, const void* b, int64_t V, int64_t E, int64_t h, int residual,
                       int act, float alpha, void* H_out, hipStream_t stream);

// fused with the aggregation its output feeds (tile plan of nt_dmpnn_tile_plan); h % 8 == 0, <= 512
bool bf16_fused_supported(int64_t h);
int launch_update_bf16_fused(const void* H, const void* S, const int64_t* src, const int64_t* rev,
                             const void* Wp, const void* b, int64_t V, int64_t E, int64_t h,
                             int residual, int act, float alpha, const int32_t* tile_ptr,
                             int64_t ntiles, const int32_t* perm, const int32_t* dsts, int reduce,
                             int aact, float aalpha, void* H_out, void* S_out, hipStream_t stream);

}  // namespace nt
