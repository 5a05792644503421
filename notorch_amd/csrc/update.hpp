// Internal interface between the nt_dmpnn_update dispatcher and its kernel variants.
#pragma once

#include <utility>

#include "common.hpp"

namespace nt {

struct UpdateArgs {
  const float* H;
  const float* S;
  const int64_t* src;
  const int64_t* rev;
  const void* Wp;   // packed fragment image (nt_dmpnn_pack_weight)
  const float* b;   // may be NULL
  int64_t V, E, h;
  int KB, NT;       // 16-deep k blocks, 16-wide column tiles
  int residual, act;
  float alpha;
  float* H_out;
  hipStream_t stream;
  // row pitches in elements (0: dense rows of h): H and S inputs, H_out and S_out outputs (fp32 fused
  // layer kernel only)
  int64_t ldi = 0, ldo = 0;
  float* S_part = nullptr;  // fused fp32: hub partial rows (row table entries < 0), see nt_dmpnn_update_fused
};

// bf16x6 fp32-emulation kernel (update_x6.hip): h % 4 == 0 and 97 <= h <= 512.
bool x6_supported(int64_t h);
size_t x6_image_bytes(int64_t h);
int pack_weight_x6(const float* W, int64_t nlayers, int64_t h, int64_t layer_stride_bytes, void* Wx,
                   hipStream_t stream);
int launch_update_x6(const UpdateArgs& a);  // a.Wp points at the x6 image

// A-stationary bf16x6 kernel (update_as.hip, 16x16x32 MFMA): h % 4 == 0, h <= 304.
bool as_supported(int64_t h);
size_t as_image_bytes(int64_t h);
int pack_weight_as(const float* W, int64_t nlayers, int64_t h, int64_t layer_stride_bytes, void* Wb,
                   hipStream_t stream);
int launch_update_as(const UpdateArgs& a);  // a.Wp points at the as16 image

// Persistent producer/consumer kernel (update_ps.hip), optionally fused with the aggregation.
bool ps_supported(int64_t h);
int launch_update_ps(const UpdateArgs& u, const int32_t* tile_ptr, int64_t ntiles,
                     const int32_t* perm, const int32_t* dsts, int reduce, int aact, float aalpha,
                     float* S_out);  // u.Wp points at the as16 image

// Persistent K-slice-ring variant (update_pk.hip): same contract as launch_update_ps.
int launch_update_pk(const UpdateArgs& u, const int32_t* tile_ptr, int64_t ntiles,
                     const int32_t* perm, const int32_t* dsts, int reduce, int aact, float aalpha,
                     float* S_out);

// fp16x3 persistent layer kernel (update_fk.hpp, built in update_pk.hip): any h % 4 == 0; tiles of
// at most fk_tile_rows(h, act, reduce, aact, fused) rows; Wimg = the fk image of the layer (header + fragment blocks).
int fk_tile_rows(int64_t h, int act, int reduce, int aact, bool fused);
int launch_update_fk(const UpdateArgs& u, const void* Wimg, const float* amax_in, float* amax_out,
                     const int32_t* tile_ptr, int64_t ntiles, int tile_rows, int max_in_degree,
                     const void* row_table, int reduce, int aact, float aalpha, float* S_out);
// fk images of nlayers separate weights (<= 16) and optionally of their transposes, one launch pair
int fk_pack_multi(const float* const* W, int64_t nlayers, int64_t h, char* const* img, char* const* imgT,
                  hipStream_t stream);
int fk_row_table(const int32_t* perm, const int32_t* dsts, const int64_t* src, const int64_t* rev, int64_t V,
                 int64_t E, void* out, hipStream_t stream);
int fk_pack(const float* W, int64_t nlayers, int64_t h, int64_t w_stride, int64_t img_stride, void* img,
            hipStream_t stream);
int fk_absmax(const float* X, int64_t n, float* out, hipStream_t stream);
// the caller's 2-float workspace ws := (max|H|, max|S|) on `stream` (H or S may be NULL: that entry is 0)
int amax_fill(float* ws, const float* H, int64_t nh, const float* S, int64_t ns, hipStream_t stream);
// bf16 storage on the same skeleton (PREC = 1): h % 8 == 0, h <= 512, tiles of <= 128 rows, Wimg =
// the bf16 fragment image; S_out / the row table exactly with a tile plan
bool fkb_supported(int64_t h);
int bf16_kernel_env();  // NT_BF16_KERNEL, read once: 0 default, 1 fk, 2 fk4
// the one-wave-per-SIMD fused walk (update_fw_kernel) takes this fused layer (128-row plans)
bool fw_active(int64_t h, int dtype, int act, int reduce, int aact);
int launch_update_fk_bf16(const UpdateArgs& u, const void* Wimg, const int32_t* tile_ptr, int64_t ntiles,
                          int tile_rows, int max_in_degree, const void* row_table, int reduce, int aact,
                          float aalpha, void* S_out);
inline int64_t fk_image_bytes(int64_t h) { return 256 + ((h + 31) / 32) * ((h + 15) / 16) * 2 * 1024; }

// Deeper-ring variant (S/H 2 chunks ahead); requires additionally NT <= 24.
int launch_update_ring(const UpdateArgs& a);

}  // namespace nt
