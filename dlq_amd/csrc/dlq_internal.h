// dlq_internal.h -- shared declarations between the HIP kernels (kernels.hip)
// and the host side (capi.cpp, resnet18.cpp, mlp.cpp).  Not installed.
#pragma once
#include <atomic>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace dlq {

// Host-side knobs behind dlq_set_knob (capi.cpp): initialised once from the
// environment when the library loads, never read from it on the hot path.
extern std::atomic<int> g_knob_l1_grid, g_knob_head_split, g_knob_graph, g_knob_gemm_tile, g_knob_ds_split,
    g_knob_prefetch, g_knob_gap_epi;
extern std::atomic<unsigned> g_knob_gen;


// Weight regions of the NEXT launch of a forward, read (into the memory-side
// cache and L2) by the current launch's last stage so that the next launch's
// first stages do not start from HBM: up to two regions of n blocks of len
// bytes (a multiple of 1 KiB), stride bytes apart.  p == nullptr: none.
struct Prefetch {
  const void* p[2];
  int n[2], stride[2], len[2];
};

// Conv launch parameters (device view).  Activations are NHWC int8.
struct ConvArgs {
  const int8_t* x;      // [N][H][W][C]
  const int8_t* w;      // packed [OCp][K]
  const float* alpha;   // [OCp]
  const float* beta;    // [OCp]
  const int8_t* res;    // [N][OH][OW][OC] or nullptr
  void* y;              // [N][OH][OW][OC] (int8 / fp32 / int32)
  float s_res;  // residual scale in output-grid units
  int N, H, W, C;
  int OH, OW, OC, OCp, K;
  int kH, kW, sH, sW, pH, pW;
  int P;     // N*OH*OW
  int relu;
  int out_kind;
  int dbg;  // ablation bits, read only by DLQ_ABLATION probe builds (tools/probe): 2 skip DMA, 4 skip epilogue
  // Downsample residual of a downsampling block's conv2 (conv3x3i.hip, int8):
  // the block input and the 1x1/s2 downsample, computed and requantised in
  // conv2's epilogue; its int8 value is the residual (res == nullptr then).
  const int8_t* ds_x;     // block input [N][2*OH][2*OW][ds_C], or nullptr
  const int8_t* ds_w;     // downsample_pack image [OCp/128][ds_C/32][128][48]
  const float* ds_alpha;  // [OCp], the downsample's output-grid units
  const float* ds_beta;
  int ds_C;
  Prefetch pf;  // the next launch's first weight blocks (engine forwards only)
  // The network's last conv (layer4.1 conv2, 7x7x512): its int8 output's
  // global average pool computed per item right after the item's epilogue
  // (conv3x3i.hip GAP): gap_y[N][512] int8 = clamp(rne(float(sum) * gap_k)).
  int8_t* gap_y;
  float gap_k;
};

// Timing-ablation switches exist only in probe builds (tools/probe/*.hip
// define DLQ_ABLATION before including a kernel source); in libdlq.so every
// DLQ_ABL() is the constant false, so no input can make a shipped kernel skip
// work or a barrier.
#ifdef DLQ_ABLATION
#define DLQ_ABL(a, bit) (((a).dbg & (bit)) != 0)
#else
#define DLQ_ABL(a, bit) false
#endif

// Stem packing: C == 4, 7x7 taps padded to 8x8 -> K = 256.
// Largest batch an engine may prepare: the conv kernels compute activation
// offsets as int ((n*H + h)*W + w)*C (layer1's 200,704 B per image at
// 8192 images is 1.64e9 < 2^31; tools/check/dma_plan.py proves the bound).
constexpr int kMaxBatch = 8192;
constexpr int kStemC = 4;
constexpr int kStemK = 8 * 8 * 4;

// output channels of a packed weight image (64, or a multiple of 128): the
// one definition every launcher, packer and test library shares
inline int packed_oc(int OC) { return OC <= 64 ? 64 : (OC + 127) / 128 * 128; }
bool is_stem(int C, int kH, int kW);

// Kernel launchers (kernels.hip, conv3x3.hip).  Return hipError_t of the launch.
hipError_t launch_conv(const ConvArgs& a, hipStream_t s);
bool conv3x3s1_supported(const ConvArgs& a);
hipError_t launch_conv3x3s1(const ConvArgs& a, hipStream_t s);
// Wide stride-1 3x3 convs: the shapes, the weight image (wpack.cpp) and the
// 392-px item kernel (conv3x3i.hip).
bool conv3x3w_shape(int C, int OC, int H, int W, int kH, int kW, int sH, int sW, int pH, int pW);
size_t conv3x3w_packed_bytes(int OC, int C);
void conv3x3w_pack(const int8_t* q_oihw, int OC, int IC, int C, int8_t* out);
hipError_t launch_conv3x3i(const ConvArgs& a, hipStream_t s);
// A downsampling block's conv2 with its 1x1/s2 downsample as the residual
// (a.ds_*; int8, ReLU, a.res == nullptr): conv3x3i_kernel<..., DSR>.
hipError_t launch_conv3x3i_dsr(const ConvArgs& a, hipStream_t s);
// Stride-2 3x3 convs: the shapes and the 1x1/s2 downsample image (wpack.cpp),
// conv1 in the wide image, and the 196-px item kernel (conv3x3s2i.hip) with
// the optional fused downsample (w_ds == nullptr: conv only).
bool conv3x3s2_shape(int C, int OC, int H, int W, int kH, int kW, int sH, int sW, int pH, int pW);
size_t downsample_packed_bytes(int OC, int C);
void downsample_pack(const int8_t* q_oc_ic, int OC, int IC, int C, int8_t* out);
hipError_t launch_conv3x3s2i(const ConvArgs& a, const int8_t* w_ds, const float* alpha_ds, const float* beta_ds,
                             int8_t* y_ds, hipStream_t s);
// Fused layer1 basic block (block_l1.hip): C == OC == 64 at 56x56, identity
// skip; generic packed weights of both convs.
bool block_l1_shape(int C, int OC, int H, int W);
hipError_t launch_block_l1(const int8_t* x, int N, const int8_t* w1, const float* a1, const float* b1,
                           const int8_t* w2, const float* a2, const float* b2, float s_res, int8_t* y,
                           hipStream_t s, bool f8 = false, const struct Prefetch* pf = nullptr);
// Fused stem (stem.hip): quantise + conv1 7x7/s2 + BN/ReLU/requant + maxpool.
size_t stem_packed_bytes();
void pack_stem_weights(const int8_t* q_oihw, const float* alpha, int8_t* out, float* alpha_abs);
hipError_t launch_stem_fused(const float* x, int N, const int8_t* w, const float* alpha, const float* beta,
                             float inv_s, int8_t* y, hipStream_t s, bool f8 = false,
                             const struct Prefetch* pf = nullptr);
void pack_stem_weights_f8(const uint8_t* q_oihw, const float* alpha, uint8_t* out, float* alpha_abs);
hipError_t launch_quantize_nchw_to_nhwc(const float* x, int N, int C, int H, int W, int Cout,
                                        float inv_s, int8_t* y, hipStream_t s);
hipError_t launch_quantize_rows(const float* x, int rows, int cols, int ldy, float inv_s,
                                int8_t* y, hipStream_t s);
hipError_t launch_maxpool(const int8_t* x, int N, int C, int H, int W, int8_t* y, hipStream_t s);
hipError_t launch_gap(const int8_t* x, int N, int C, int HW, float k, int8_t* y, hipStream_t s);   // C % 16 == 0
hipError_t launch_gap4(const int8_t* x, int N, int C, int HW, float k, int8_t* y, hipStream_t s);  // C % 4 == 0
hipError_t launch_linear(const int8_t* x, int N, int K, const int8_t* w, int OC, const float* alpha,
                         const float* beta, int relu, int out_kind, void* y, hipStream_t s);
// One-launch int8 MLP (quantise -> fc1 + bias + ReLU + requant -> fc2 + bias), head.hip.
hipError_t launch_mlp_fused(const float* x, int N, int in, int kp, float inv_s, const int8_t* w1, int H,
                            const float* a1, const float* b1, const int8_t* w2, int OC, const float* a2,
                            const float* b2, int8_t* hq, float* y, hipStream_t s, int mr = 0);
// false: the fused kernel's LDS (rows, hidden layer, alpha/beta) exceeds 64 KiB
// for this shape; dlq_mlp_forward then runs quantize_rows + two linear launches.
bool mlp_fused_fits(int kp, int H, int OC, int mr = 0);
hipError_t launch_gap_fc(const int8_t* x, int N, int C, int HW, float k, const int8_t* w, int OC,
                         const float* alpha, const float* beta, float* y, hipStream_t s);  // C == 512, HW <= 56
// dlq_gemm_s8s8s32 (gemm.hip): row-major int8 A[M][K] . B[K][N] -> int32 C.
hipError_t launch_gemm_s8s8s32(const int8_t* A, const int8_t* B, int32_t* C, int M, int N, int K, hipStream_t s);
// dlq_gemm_s8s8s32_nt (gemm.hip): the same with B supplied as Bt[N][K].
hipError_t launch_gemm_s8s8s32_nt(const int8_t* A, const int8_t* Bt, int32_t* C, int M, int N, int K, hipStream_t s);
hipError_t launch_im2col_nchw(const int8_t* x, int N, int C, int H, int W, int kH, int kW, int sH,
                              int sW, int pH, int pW, int8_t* col, hipStream_t s);

// fp8 (e4m3) path (kernels.hip conv_s8_kernel<..., F8>, fp8.hip): generic
// packed layout only.
hipError_t launch_conv_f8(const ConvArgs& a, hipStream_t s);
// conv3x3i with e4m3 operands (wide stride-1 shapes, conv3x3w_pack image).
hipError_t launch_conv3x3i_f8(const ConvArgs& a, hipStream_t s);
// conv3x3s2i with e4m3 operands (+ the fused 1x1/s2 downsample when w_ds).
hipError_t launch_conv3x3s2i_f8(const ConvArgs& a, const uint8_t* w_ds, const float* alpha_ds, const float* beta_ds,
                                uint8_t* y_ds, hipStream_t s);
// fp8 weight image choice: the wide layout for conv3x3w_shape and
// conv3x3s2_shape, else generic.
bool f8_wide(int C, int OC, int H, int W, int kH, int kW, int sH, int sW, int pH, int pW);
size_t packed_bytes_f8(int C, int OC, int H, int W, int kH, int kW, int sH, int sW, int pH, int pW);
void pack_conv_weights_f8(int C, int OC, int H, int W, int kH, int kW, int sH, int sW, int pH, int pW,
                          const uint8_t* q_oihw, int IC, uint8_t* packed);
uint8_t f8_encode_host(float y);
uint8_t f8_requant_host(float y, float lo);
void quantize_weights_f8(const float* w, int OC, int K, uint8_t* q, float* scale);

// Reference-semantics fp32 ops (ref_f32.hip; oracle.c ora_*_f32 bit for bit),
// NCHW over B images.  amax (nullable): device uint, max |output| as float bits.
hipError_t launch_ref_conv_bn(const float* x, int B, int IC, int H, int W, const float* w, int OC, int k, int s, int p,
                              const float* g, const float* b, const float* m, const float* d, int relu, float* y,
                              unsigned* amax, hipStream_t st);
hipError_t launch_ref_add_relu(float* y, const float* skip, long n, unsigned* amax, hipStream_t st);
hipError_t launch_ref_maxpool(const float* x, int NC, int H, int W, float* y, hipStream_t st);
hipError_t launch_ref_gap(const float* x, int NC, int HW, float* y, unsigned* amax, hipStream_t st);
hipError_t launch_ref_fc(const float* g, int B, const float* W, const float* bias, int O, int I, float* out,
                         hipStream_t st);
hipError_t launch_amax(const float* x, long n, unsigned* amax, hipStream_t st);

// Thread-local error message (capi.cpp).
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

// Host weight preparation (capi.cpp), identical op order to oracle/oracle.c.
void quantize_weights(const float* w, int OC, int K, int8_t* q, float* scale);
void fold_bn(float s_x, const float* s_w, const float* g, const float* b, const float* m,
             const float* v, float eps, float s_y, int OC, float* alpha, float* beta);
float res_scale(float s_r, float s_y);
// Generic / stem layouts (any shape the v1 kernel runs), and the
// shape-selected image dlq_conv2d_nhwc_s8 expects (may be the wide layout).
size_t packed_bytes(int OC, int C, int kH, int kW);
void pack_conv_weights(const int8_t* q_oihw, int OC, int IC, int kH, int kW, int C,
                       int8_t* packed);
bool wide_layout(int C, int OC, int H, int W, int kH, int kW, int sH, int sW, int pH, int pW);
size_t packed_bytes_for(int C, int OC, int H, int W, int kH, int kW, int sH, int sW, int pH, int pW);
void pack_conv_weights_for(int C, int OC, int H, int W, int kH, int kW, int sH, int sW, int pH, int pW,
                           const int8_t* q_oihw, int IC, int8_t* packed);

// Validation + ConvArgs of one conv launch (capi.cpp conv_args).
}  // namespace dlq
struct dlq_conv_desc;
namespace dlq {
int conv_args_checked(const dlq_conv_desc* d, const int8_t* x, const int8_t* w_packed, const float* alpha,
                      const float* beta, const int8_t* residual, float res_scale, int relu, int out_kind, void* y,
                      ConvArgs& a);
// dlq_conv2d_nhwc_s8 / dlq_conv2d_s2_ds_nhwc_s8 with the next launch's weight
// regions (Prefetch; nullptr = none) for the engine's forward.
// gap_y: the wide 7x7x512 conv also writes its output's int8 GAP codes
// (ConvArgs::gap_y / gap_k; the network's last conv only).
int conv2d_nhwc_s8_pf(const dlq_conv_desc* d, const int8_t* x, const int8_t* w_packed, const float* alpha,
                      const float* beta, const int8_t* residual, float res_scale, int relu, int out_kind, void* y,
                      void* stream, const Prefetch* pf, int8_t* gap_y = nullptr, float gap_k = 0.f);
int conv2d_s2_ds_nhwc_s8_pf(const dlq_conv_desc* d, const int8_t* x, const int8_t* w_packed, const float* alpha,
                            const float* beta, const int8_t* w_ds, const float* alpha_ds, const float* beta_ds,
                            int8_t* y, int8_t* y_ds, void* stream, const Prefetch* pf);

inline int out_dim(int in, int k, int s, int p) { return (in + 2 * p - k) / s + 1; }

}  // namespace dlq
