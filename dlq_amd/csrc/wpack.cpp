// wpack.cpp -- host-side weight images of the wide conv kernels (conv3x3i.hip,
// conv3x3s2i.hip) and the shapes they run.  Host code only: the kernels read
// these bytes verbatim by LDS-DMA, one 32-channel slice per ring stage.
//
// Source layout is the reference's OIHW (CUDA/resnet18-kernel-lab/cpp/fp32/
// runtime/infer_e2e.cu:102-136 reads Wk[OC][IC][kH][kW]), quantised per output
// channel (capi.cpp quantize_weights).
#include <cstring>

#include "dlq_internal.h"

namespace dlq {

namespace {
constexpr int kSlice = 32;              // input channels per ring stage
constexpr int kTileOC = 128;            // output channels per weight block
constexpr int kPitch3 = 9 * kSlice + 16;  // 3x3 row: 9 taps x 32 B + 16 pad (304 B, odd # of 16-B units)
constexpr int kPitch1 = kSlice + 16;      // 1x1 downsample row (48 B, odd # of 16-B units)
}  // namespace

bool conv3x3w_shape(int C, int OC, int H, int W, int kH, int kW, int sH, int sW, int pH, int pW) {
  if (!(kH == 3 && kW == 3 && sH == 1 && sW == 1 && pH == 1 && pW == 1 && H == W && OC == C)) return false;
  return (W == 28 && C == 128) || (W == 14 && C == 256) || (W == 7 && C == 512);
}

bool conv3x3s2_shape(int C, int OC, int H, int W, int kH, int kW, int sH, int sW, int pH, int pW) {
  if (!(kH == 3 && kW == 3 && sH == 2 && sW == 2 && pH == 1 && pW == 1 && H == W && OC == 2 * C)) return false;
  return (W == 56 && C == 64) || (W == 28 && C == 128) || (W == 14 && C == 256);
}

size_t conv3x3w_packed_bytes(int OC, int C) { return (size_t)packed_oc(OC) * (C / kSlice) * kPitch3; }

// OIHW q[OC][IC][3][3] -> [OCp/128][C/32][128 oc][9 taps x 32 channels + 16 pad]
void conv3x3w_pack(const int8_t* q, int OC, int IC, int C, int8_t* out) {
  std::memset(out, 0, conv3x3w_packed_bytes(OC, C));
  const int NS = C / kSlice;
  for (int o = 0; o < OC; ++o)
    for (int c = 0; c < IC; ++c)
      for (int t = 0; t < 9; ++t) {
        const int ot = o / kTileOC, ol = o % kTileOC, j = c / kSlice, cc = c % kSlice;
        out[(((size_t)ot * NS + j) * kTileOC + ol) * kPitch3 + t * kSlice + cc] = q[((size_t)o * IC + c) * 9 + t];
      }
}

size_t downsample_packed_bytes(int OC, int C) { return (size_t)packed_oc(OC) * (C / kSlice) * kPitch1; }

// 1x1 weights q[OC][IC] -> [OCp/128][C/32][128 oc][32 channels + 16 zero]
void downsample_pack(const int8_t* q, int OC, int IC, int C, int8_t* out) {
  std::memset(out, 0, downsample_packed_bytes(OC, C));
  const int NS = C / kSlice;
  for (int o = 0; o < OC; ++o)
    for (int c = 0; c < IC; ++c) {
      const int ot = o / kTileOC, ol = o % kTileOC, j = c / kSlice, cc = c % kSlice;
      out[(((size_t)ot * NS + j) * kTileOC + ol) * kPitch1 + cc] = q[(size_t)o * IC + c];
    }
}

}  // namespace dlq
