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
};

// LDS-DMA streamed fp32 MFMA kernel (update_glds.hip); requires h % 4 == 0, NT <= 32, 16-B aligned
// H, S, H_out, b.
int launch_update_glds(const UpdateArgs& a);

}  // namespace nt
