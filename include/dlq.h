/*
 * dlq.h -- C ABI of the MI355X-native int8 CNN inference path (libdlq.so).
 *
 * Drop-in for the conv/GEMM inference path of yeontachi/DLQ:
 *   CUDA/resnet18-kernel-lab/cpp/fp32/{kernels,runtime}  (ResNet-18)
 *   CUDA/MNIST_on_GPU/v4.cu, v5.cu                      (MLP FC GEMM, forward)
 * Every entry point below names the reference interface it replaces
 * (file:line, relative to the reference repository root; "RK" abbreviates
 * CUDA/resnet18-kernel-lab/cpp/fp32).
 *
 * Conventions (differences from the reference are deliberate):
 *   - plain C types only; device pointers are HIP device addresses; `stream`
 *     is a hipStream_t (NULL = the legacy default stream, as in the reference);
 *   - every call returns an int status (DLQ_OK = 0) and NEVER exits the
 *     process (the reference's CUDA_CHECK calls std::exit(1), RK/runtime/
 *     utils.hpp:23-32); dlq_last_error() gives the message of the last failure
 *     on the calling thread;
 *   - the batch dimension N is honoured everywhere (the reference hard-wires
 *     N=1, RK/kernels/im2col.cu:11-12);
 *   - activations are int8 NHWC on the device ("channels-last", the layout the
 *     int8 MFMA contraction wants); NCHW survives at the boundaries: the fp32
 *     input is NCHW (as RK/runtime/infer_e2e.cu:254-256), and
 *     dlq_im2col_nchw_s8 / stage dumps use NCHW.
 * No call allocates or synchronises unless documented (the create / prepare
 * calls do), so forward calls can be captured into a hipGraph.
 */
#ifndef DLQ_H
#define DLQ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DLQ_OK 0
#define DLQ_ERR_ARG 1    /* bad shape / pointer / unsupported configuration      */
#define DLQ_ERR_HIP 2    /* HIP runtime error (utils.hpp:23-32 analogue)          */
#define DLQ_ERR_LAUNCH 3 /* kernel launch failed (utils.hpp:34-45 returns 3)     */
#define DLQ_ERR_IO 4     /* file I/O (utils.hpp:48-67 analogue)                   */
#define DLQ_ERR_STATE 5  /* object used before prepare / missing tensor or scale */

/* Epilogue output kinds of dlq_conv2d_nhwc_s8 / dlq_linear_s8. */
#define DLQ_OUT_S8 0  /* requantised int8 (fused BN/bias, residual, ReLU)         */
#define DLQ_OUT_F32 1 /* fp32 = fmaf(float(acc), alpha, beta) (dequant / logits) */
#define DLQ_OUT_S32 2 /* raw int32 accumulators (parity / debugging)             */

const char* dlq_version(void);
const char* dlq_last_error(void);
/* Name of HIP device `dev` (e.g. "gfx950"); DLQ_ERR_HIP without a GPU. */
int dlq_device_arch(int dev, char* buf, int buflen);

/* ------------------------------------------------------------------------ */
/* Host-side weight preparation (no device, deterministic, bit-identical to */
/* the CPU oracle).  The reference copies fp32 OIHW weights as-is           */
/* (RK/runtime/infer_e2e.cu:114-126 is an identity repack).                 */
/* ------------------------------------------------------------------------ */

/* Symmetric per-output-channel quantisation of w[OC][K]:
 * scale[o] = max|w[o,:]|/127 (1 if all zero), q = clamp(rne(w/scale), +-127). */
int dlq_quantize_weights_s8(const float* w, int OC, int K, int8_t* q, float* scale);

/* Dequant * BatchNorm * requant folded into one affine per channel, in units
 * of the output int8 grid (replaces bn_launch, RK/runtime/infer_e2e.cu:83-97
 * and RK/kernels/bn_inference.cu:22-27):
 *   t = g/sqrtf(v+eps); inv = 1/s_y;
 *   alpha = ((s_x*s_w)*t)*inv; beta = (b - m*t)*inv.                        */
int dlq_fold_bn(float s_x, const float* s_w, const float* g, const float* b, const float* m,
                const float* v, float eps, float s_y, int OC, float* alpha, float* beta);
/* A residual of scale s_r added into an output of scale s_y: s_r*(1/s_y). */
float dlq_res_scale(float s_r, float s_y);

/* Padded output-channel count the packed weights / alpha / beta must have. */
int dlq_conv_packed_oc(int OC);

typedef struct dlq_conv_desc {
  int N, H, W, C; /* input NHWC; C = stored channels (4 for the RGB stem)     */
  int OC;         /* output channels                                          */
  int kH, kW, sH, sW, pH, pW;
} dlq_conv_desc;

/* Bytes of the packed weight image for the conv `d` (N is ignored).  The
 * image is specific to the descriptor, like a cuDNN filter transform: the
 * kernel that dlq_conv2d_nhwc_s8 selects for `d` reads exactly this layout.
 * Supported: C % 64 == 0 (any kH, kW), the stem (C == 4, 7x7), and C % 32 ==
 * 0 for the wide stride-1 3x3 convs.  Returns 0 for unsupported shapes.
 * Layouts (q = OIHW int8):
 *  - wide 3x3: stride 1 (C == OC in {128 @28x28, 256 @14x14, 512 @7x7}, p1)
 *    and stride 2 (C -> 2C at 56x56x64, 28x28x128, 14x14x256, p1):
 *      [OCp/128][C/32][128 oc][9 taps x 32 channels + 16 zero bytes]
 *    one contiguous 38,912-byte block per (128-oc tile, 32-channel slice),
 *    copied verbatim into LDS (row pitch 304 B: conflict-free ds_read_b128);
 *  - stem (C == 4, 7x7): [OCp][8][8][4], taps padded to 8x8;
 *  - otherwise (C % 64 == 0): [C/64][OCp/64][64 oc][kH*kW taps][4 x 16 B]
 *    with the 4 chunks of a 64-byte tap row stored at chunk ^ ((oc%64>>2)&3). */
size_t dlq_conv_packed_bytes(const dlq_conv_desc* d);
/* Pack q_oihw[OC][IC][kH][kW] (IC <= C; channels IC..C-1 and padded output
 * rows are zero) into the image dlq_conv_packed_bytes(d) describes. */
int dlq_pack_conv_weights_s8(const dlq_conv_desc* d, const int8_t* q_oihw, int IC, int8_t* packed);

/* ------------------------------------------------------------------------ */
/* Per-layer C-ABI in the reference's layout (layerops.hip).  These mirror   */
/* the reference's extern "C" kernels and host helpers (RK/include/          */
/* utils.hpp:74-82, RK/runtime/infer_e2e.cu:64-219): same argument order,    */
/* NCHW / OIHW / row-major operands, batch honoured, explicit stream, int    */
/* status.  The NHWC operators further below are the fast path.              */
/* ------------------------------------------------------------------------ */

/* Process-wide test / A-B knobs, read on the host at each forward without
 * touching the environment (each starts from its environment variable,
 * read ONCE when the library loads; no reference counterpart):
 *   "l1_grid"    (DLQ_L1_GRID)    cap on the layer1 block's grid, 0 = one
 *                                 workgroup per CU (>0 puts several images in
 *                                 one workgroup);
 *   "head_split" (DLQ_HEAD_SPLIT) 1 = GAP and FC as two launches;
 *   "graph"      (DLQ_GRAPH)      1 = replay the forward as a hipGraph;
 *   "gemm_tile"  (DLQ_GEMM_TILE)  dlq_gemm_s8s8s32's tile, 0 = by shape,
 *                                 1 = 256 x 256, 2 = 256 x 128, 3 = 128 x 128,
 *                                 4 = 256 x 224, 5 = 224 x 128, 6 = 224 x 256;
 *   "ds_split"   (DLQ_DS_SPLIT)   0 = (default) the engine computes the
 *                                 layer2.0 / layer3.0 1x1/s2 downsample in
 *                                 their conv2 launch (dlq_conv2d_dsres_nhwc_s8);
 *                                 -1 = fused into the stride-2 conv1 launch
 *                                 (dlq_conv2d_s2_ds_nhwc_s8) as for layer4.0;
 *                                 1 / 2 = in conv2 for layer3.0 / layer2.0 only;
 *   "prefetch"   (DLQ_PREFETCH)   0 = (default) each launch of a forward
 *                                 reads the next launch's first weights during
 *                                 its last stage; -1 = off;
 *   "gap_epi"    (DLQ_GAP_EPI)    0 = (default) the last conv pools its own
 *                                 output and the head is the FC alone;
 *                                 -1 = the fused GAP + FC head launch.
 * Returns DLQ_ERR_ARG for an unknown name. */
int dlq_set_knob(const char* name, int value);
int dlq_get_knob(const char* name, int* value);

/* Select the device and check it is gfx950 (the kernels' only target).    */
int dlq_init(int device);
/* Synchronise the device; pairs with dlq_init.                            */
int dlq_finalize(void);
/* q[i] = clamp(rne(x[i] * inv_s), +-127): the input quantisation (new; the
 * reference feeds fp32 straight to im2col, RK/runtime/infer_e2e.cu:255-256). */
int dlq_quantize_f32_s8(const float* x, size_t n, float inv_s, int8_t* q, void* stream);
/* sgemm_tiled (RK/kernels/sgemm_tiled.cu:5-46) on int8: C[M][N] (int32) =
 * A[M][K] . B[K][N], all row-major, any M, N, K. */
int dlq_gemm_s8s8s32(const int8_t* A, const int8_t* B, int32_t* C, int M, int N, int K, void* stream);
/* The same contraction with B supplied transposed, Bt[N][K] (each output
 * column's K bytes contiguous, as the MFMA's B operand wants): C[M][N] =
 * A[M][K] . Bt^T.  New (the reference's sgemm_tiled is NN only); for callers
 * that hold the im2col panel K-contiguous, or weights as the right operand.
 * Any M, N, K; the LDS-DMA kernel needs only K % 16 == 0 and 16-byte aligned
 * A / Bt.  int32 results identical to dlq_gemm_s8s8s32 on B = Bt^T. */
int dlq_gemm_s8s8s32_nt(const int8_t* A, const int8_t* Bt, int32_t* C, int M, int N, int K, void* stream);
/* conv2d_nchw_im2col_gemm (RK/runtime/infer_e2e.cu:102-136; + bn_launch
 * :83-97 + relu) on int8: x[N][IC][H][W], w_oihw[OC][IC][kH][kW] (int8,
 * packed and uploaded per call like the reference's per-call weight copy),
 * alpha/beta[OCp] (dlq_fold_bn), out_kind DLQ_OUT_S8 (y int8 NCHW) or
 * DLQ_OUT_S32 (y int32 NCHW accumulators).  *OH, *OW as the reference
 * returns them.  workspace >= dlq_conv2d_nchw_workspace_bytes(...) device
 * bytes.  Shapes: those dlq_conv2d_nhwc_s8 supports (IC % 64 == 0, the RGB
 * stem, the wide 3x3 convs). */
size_t dlq_conv2d_nchw_workspace_bytes(int N, int IC, int H, int W, int OC, int kH, int kW, int sH, int sW, int pH,
                                       int pW);
int dlq_conv2d_nchw_s8(const int8_t* x, int N, int IC, int H, int W, const int8_t* w_oihw, int OC, int kH, int kW,
                       int sH, int sW, int pH, int pW, const float* alpha, const float* beta, int relu, int out_kind,
                       void* y, void* workspace, size_t ws_bytes, void* stream, int* OH, int* OW);
/* bn_inference + relu_forward (RK/kernels/bn_inference.cu:5-28, relu.cu:4-10)
 * as the standalone requantising epilogue: y = clamp(rne(fma(acc, alpha[c],
 * beta[c])), relu ? 0 : -127, 127) on NCHW [N][C][HW]. */
int dlq_bn_relu_requant_s8(const int32_t* acc, int N, int C, int HW, const float* alpha, const float* beta, int relu,
                           int8_t* y, void* stream);
/* add_inplace + relu_forward (RK/kernels/add.cu:2-8) in the int8 domain:
 * y = clamp(rne(fma(r, r_scale, a * a_scale)), relu ? 0 : -127, 127), with
 * a_scale = s_a/s_y, r_scale = s_r/s_y (output-grid units). */
int dlq_add_relu_requant_s8(const int8_t* a, const int8_t* r, size_t n, float a_scale, float r_scale, int relu,
                            int8_t* y, void* stream);
/* maxpool2d_3x3_s2p1_nchw (RK/kernels/maxpool2d.cu:4-41) on int8 NCHW. */
int dlq_maxpool2d_3x3_s2p1_nchw_s8(const int8_t* x, int N, int C, int H, int W, int8_t* y, void* stream);
/* gap_global (RK/kernels/gap_global.cu:2-33) on int8 NCHW [N][C][HW] ->
 * int8 [N][C]: exact int32 sum, clamp(rne(float(sum) * k)). */
int dlq_gap_s8(const int8_t* x, int N, int C, int HW, float k, int8_t* y, void* stream);
/* fc_forward (RK/runtime/infer_e2e.cu:206-219, bias on the device):
 * logits[N][OC] = fma(acc, alpha, bias) = dlq_linear_s8(..., DLQ_OUT_F32). */
int dlq_fc_s8(const int8_t* g, int N, int K, const int8_t* w_packed, int OC, const float* alpha, const float* bias,
              float* logits, void* stream);
/* y = float(acc) * scale[c] on NCHW [N][C][HW] (int32 -> fp32 dequant). */
int dlq_dequant_s32_f32(const int32_t* acc, int N, int C, int HW, const float* scale, float* y, void* stream);

/* ------------------------------------------------------------------------ */
/* Device operators (per-layer entry points; all asynchronous on `stream`)  */
/* ------------------------------------------------------------------------ */

/* Input quantisation (new; the reference feeds fp32 straight to im2col,
 * RK/runtime/infer_e2e.cu:255-256): fp32 NCHW x[N][C][H][W] ->
 * int8 NHWC y[N][H][W][Cout], channels C..Cout-1 zero; q = clamp(rne(x*inv_s)). */
int dlq_quantize_nchw_to_nhwc_s8(const float* x, int N, int C, int H, int W, int Cout, float inv_s,
                                 int8_t* y, void* stream);
/* Row quantisation fp32 x[rows][cols] -> int8 y[rows][ldy] (zero padded). */
int dlq_quantize_rows_s8(const float* x, int rows, int cols, int ldy, float inv_s, int8_t* y,
                         void* stream);

/* Implicit-im2col int8 conv + fused epilogue.  Replaces
 * conv2d_nchw_im2col_gemm (RK/runtime/infer_e2e.cu:102-136: im2col_nchw +
 * sgemm_tiled) followed by bn_launch (:83-97), add_inplace (RK/kernels/add.cu)
 * and relu_forward (RK/kernels/relu.cu) as wired in basic_block_forward
 * (:156-203).  Output NHWC [N][OH][OW][OC]:
 *   DLQ_OUT_S8 : alpha/beta/res_scale in output-grid units (dlq_fold_bn,
 *                dlq_res_scale):
 *                y = fmaf(float(acc), alpha[o], beta[o]);
 *                y = fmaf(float(residual), res_scale, y) if residual != NULL;
 *                out = rne(clamp(y, relu ? 0 : -127, 127))
 *   DLQ_OUT_F32: out = fmaf(float(acc), alpha[o], beta[o]) (max(.,0) if relu)
 *   DLQ_OUT_S32: out = acc (int32)                                           */
int dlq_conv2d_nhwc_s8(const dlq_conv_desc* d, const int8_t* x, const int8_t* w_packed,
                       const float* alpha, const float* beta, const int8_t* residual,
                       float res_scale, int relu, int out_kind, void* y, void* stream);

/* Downsampling BasicBlock front (infer_e2e.cu:161-176 conv1 + bn + relu and
 * :187-196 the 1x1/s2 downsample conv + bn) in one launch: the 3x3/s2/p1
 * conv (C -> 2C; weights packed by dlq_pack_conv_weights_s8 for `d`) ->
 * alpha/beta -> ReLU -> int8 y, and the 1x1/s2 conv of the same input
 * (weights q_ds[OC][IC] packed by dlq_pack_downsample_weights_s8 as
 * [OCp/128][C/32][128][32 + 16 zero]) -> alpha_ds/beta_ds -> int8 y_ds (no
 * ReLU).  Both in output-grid units (dlq_fold_bn).  Supported for the
 * ResNet-18 shapes 56x56x64, 28x28x128 and 14x14x256 (NHWC input).  Results
 * equal two dlq_conv2d_nhwc_s8 calls (3x3/s2 with relu, 1x1/s2 without). */
size_t dlq_downsample_packed_bytes(int OC, int C);
int dlq_pack_downsample_weights_s8(const int8_t* q_ds, int OC, int IC, int C, int8_t* packed);
int dlq_conv2d_s2_ds_nhwc_s8(const dlq_conv_desc* d, const int8_t* x, const int8_t* w_packed,
                             const float* alpha, const float* beta, const int8_t* w_ds, const float* alpha_ds,
                             const float* beta_ds, int8_t* y, int8_t* y_ds, void* stream);

/* Downsampling BasicBlock back (infer_e2e.cu:177-186 conv2 + bn, :187-196
 * the 1x1/s2 downsample conv + bn, :197-202 add + relu) in one launch: the
 * 3x3/s1/p1 conv of h (d: C == OC, the layer2/3 shapes 28x28x128 and
 * 14x14x256; w_packed from dlq_pack_conv_weights_s8) -> alpha/beta, plus the
 * residual r = the block input x_blk[N][2H][2W][C/2]'s 1x1/s2 downsample
 * (w_ds from dlq_pack_downsample_weights_s8, alpha_ds/beta_ds) requantised to
 * int8 exactly as dlq_conv2d_s2_ds_nhwc_s8 stores y_ds, times res_scale ->
 * ReLU -> int8 y.  Equals dlq_conv2d_s2_ds_nhwc_s8's y_ds fed to
 * dlq_conv2d_nhwc_s8 as the residual, bit for bit; the downsample's output
 * never goes to memory. */
int dlq_conv2d_dsres_nhwc_s8(const dlq_conv_desc* d, const int8_t* h, const int8_t* w_packed, const float* alpha,
                             const float* beta, const int8_t* x_blk, const int8_t* w_ds, const float* alpha_ds,
                             const float* beta_ds, float res_scale, int8_t* y, void* stream);

/* Fused layer1 basic block: int8 NHWC x[N][56][56][64] -> y (same shape) =
 * ReLU(requant(BN2(conv2(h)) + s_res * x)), h = ReLU(requant(BN1(conv1(x)))),
 * both convs 3x3/s1/p1 64->64, in ONE launch (the intermediate h stays in
 * LDS; x is read once and is also the residual).  w1, w2: images from
 * dlq_pack_conv_weights_s8 for the descriptor {N, 56, 56, 64, 64, 3, 3, 1, 1,
 * 1, 1}; alpha/beta[64] in output-grid units (dlq_fold_bn); s_res =
 * dlq_res_scale(s_x, s_y2).  Bit-identical to dlq_conv2d_nhwc_s8(conv1,
 * relu) followed by dlq_conv2d_nhwc_s8(conv2, residual x, relu).  Replaces
 * basic_block_forward (RK/runtime/infer_e2e.cu:156-203) for layer1.0/1.1. */
int dlq_block_l1_nhwc_s8(const int8_t* x, int N, const int8_t* w1, const float* alpha1, const float* beta1,
                         const int8_t* w2, const float* alpha2, const float* beta2, float s_res, int8_t* y,
                         void* stream);

/* Fused stem: fp32 NCHW x[N][3][224][224] -> int8 NHWC y[N][56][56][64] =
 * maxpool3x3s2p1(requant(ReLU(BN(conv7x7s2p3(quant(x)))))).  One launch
 * replaces the input upload + conv1 + bn1 + relu + maxpool sequence of
 * RK/runtime/infer_e2e.cu:255-293; the 112x112 conv1 output never reaches
 * HBM.  dlq_pack_stem_weights_s8 turns the int8 OIHW conv1 weights and conv1's
 * alpha[64] (output-grid units, dlq_fold_bn) into the kernel's image (64 x
 * 256 B: 7x7x3 taps re-indexed for a 2x2 space-to-depth input; rows of
 * channels with alpha < 0 negated) and alpha_packed = |alpha|; pass
 * alpha_packed and the unchanged beta[64] to dlq_stem_fused_s8 (inv_s =
 * 1/input scale).  Bit-identical to dlq_quantize_nchw_to_nhwc_s8 +
 * dlq_conv2d_nhwc_s8 (stem, alpha/beta) + dlq_maxpool2d_3x3_s2p1_nhwc_s8. */
size_t dlq_stem_packed_bytes(void);
int dlq_pack_stem_weights_s8(const int8_t* q_oihw, const float* alpha, int8_t* packed, float* alpha_packed);
int dlq_stem_fused_s8(const float* x, int N, const int8_t* w_stem, const float* alpha, const float* beta,
                      float inv_s, int8_t* y, void* stream);

/* Dense layer on int8 rows: y[N][OC] from x[N][K] (K % 64 == 0) and weights
 * packed as the 1x1 conv {H = W = 1, C = K, OC} (dlq_pack_conv_weights_s8);
 * same epilogue kinds.  Replaces fc_forward
 * (RK/runtime/infer_e2e.cu:206-219: sgemm_tiled M=1000,N=1,K=512 + host bias)
 * and the MNIST forward GEMMs (CUDA/MNIST_on_GPU/v4.cu:255-302
 * matmul_a_b_kernel + bias_forward_kernel + relu_forward_kernel;
 * v5.cu:127-157 cublasSgemm + bias_add_kernel + relu_kernel). */
int dlq_linear_s8(const int8_t* x, int N, int K, const int8_t* w_packed, int OC, const float* alpha,
                  const float* beta, int relu, int out_kind, void* y, void* stream);

/* 3x3/s2/p1 max pool on int8 NHWC (RK/kernels/maxpool2d.cu:4-41, launched at
 * RK/runtime/infer_e2e.cu:283-293; out-of-bounds taps skipped). */
int dlq_maxpool2d_3x3_s2p1_nhwc_s8(const int8_t* x, int N, int C, int H, int W, int8_t* y,
                                   void* stream);

/* Global average pool (gap_global_ref, RK/runtime/infer_e2e.cu:37-61;
 * RK/kernels/gap_global.cu) on int8 NHWC [N][HW][C] -> int8 [N][C]:
 * exact int32 sum, then clamp(rne(float(sum) * k)), k = s_in/HW/s_out. */
int dlq_gap_nhwc_s8(const int8_t* x, int N, int C, int HW, float k, int8_t* y, void* stream);

/* The network head in one launch: dlq_gap_nhwc_s8 followed by
 * dlq_linear_s8(..., relu 0, DLQ_OUT_F32) (gap_global_ref + fc_forward,
 * RK/runtime/infer_e2e.cu:417-433), bit-identical logits, the int8 GAP codes
 * kept on chip.  C must be 512 (= K) and HW <= 56 (DLQ_ERR_ARG otherwise). */
int dlq_gap_fc_s8(const int8_t* x, int N, int C, int HW, float k, const int8_t* w_packed, int OC,
                  const float* alpha, const float* beta, float* y, void* stream);

/* im2col in the reference's row order r = c*kH*kW + kh*kW + kw
 * (RK/kernels/im2col.cu:5-58) on int8 NCHW, batch honoured: col[N][K][OH*OW].
 * Parity/debug only -- the conv kernel gathers patches implicitly. */
int dlq_im2col_nchw_s8(const int8_t* x, int N, int C, int H, int W, int kH, int kW, int sH, int sW,
                       int pH, int pW, int8_t* col, void* stream);

/* ------------------------------------------------------------------------ */
/* ResNet-18 engine: the launcher's per-layer sequence (RK/runtime/         */
/* infer_e2e.cu:259-438) with weights resident and a preallocated workspace */
/* ------------------------------------------------------------------------ */
typedef struct dlq_resnet18 dlq_resnet18;

int dlq_resnet18_create(dlq_resnet18** out);
void dlq_resnet18_destroy(dlq_resnet18* m);
/* fp32 tensor by torch state_dict name, e.g. "layer1.0.conv1.weight",
 * "bn1.running_var", "fc.bias" (the export format of
 * tools/export_resnet18.py:85-104; the loader of infer_e2e.cu:226-228). */
int dlq_resnet18_set_tensor(dlq_resnet18* m, const char* name, const float* data, size_t n);
/* Activation scale (fp32, > 0) by site: "input", "conv1",
 * "layerX.Y.conv1", "layerX.Y.conv2", "layerX.0.downsample", "gap". */
int dlq_resnet18_set_scale(dlq_resnet18* m, const char* name, float scale);
/* Read every tensor from <dir>/<name>.bin (the reference's manifest dir,
 * RK/runtime/infer_e2e.cu:262-334,428-429). */
int dlq_resnet18_load_manifest(dlq_resnet18* m, const char* dir);
/* Pre-quantised weight of a conv / fc layer (int8 manifest): int8 [n] in the
 * fp32 tensor's layout, per-output-channel scales [n_scale = OC], values in
 * +-127.  Replaces the fp32 copy; prepare then skips quantisation (the same
 * bytes as quantising the fp32 weight with dlq_quantize_weights_s8). */
int dlq_resnet18_set_tensor_s8(dlq_resnet18* m, const char* name, const int8_t* q, size_t n, const float* scale,
                               size_t n_scale);
/* Write the model's tensors as a manifest directory in the reference's
 * export format (tools/export_resnet18.py:57-113: <name>.bin raw tensors +
 * manifest.json with shape / layout / kind / path).  int8 = 1: conv and fc
 * weights as int8 <name>.bin + fp32 <name>.scale.bin, "dtype": "int8"
 * (dlq_resnet18_load_manifest reads both kinds). */
int dlq_resnet18_save_manifest(const dlq_resnet18* m, const char* dir, int int8);
/* Write the activation scales in dlq_resnet18_load_scales' text format. */
int dlq_resnet18_save_scales(const dlq_resnet18* m, const char* path);
/* Read "<site> <scale>" lines (the int8 quant block). */
int dlq_resnet18_load_scales(dlq_resnet18* m, const char* path);
/* Quantise + fold + upload weights, allocate the workspace for up to
 * max_batch images.  Synchronous. */
int dlq_resnet18_prepare(dlq_resnet18* m, int max_batch, void* stream);
/* logits[B][1000] fp32 (device) from x[B][3][224][224] fp32 NCHW (device). */
int dlq_resnet18_forward(dlq_resnet18* m, const float* x, int B, float* logits, void* stream);
/* basic_block_forward (RK/runtime/infer_e2e.cu:139-203) of block 0..7
 * (layer1.0 .. layer4.1) of a prepared model on int8 NHWC x (scale of the
 * block input) -> int8 NHWC y (scale of the block's conv2); intermediates
 * live in the model's workspace (do not overlap with a forward). */
int dlq_basic_block_s8(dlq_resnet18* m, int block, const int8_t* x, int N, int8_t* y, void* stream);
/* Keep snapshots of every stage output (for dumps/parity; costs D2D copies
 * inside forward).  Takes effect at the next dlq_resnet18_prepare. */
int dlq_resnet18_set_keep_stages(dlq_resnet18* m, int on);
/* Copy a stage activation of the last forward to device memory `dst`:
 * "stem_pool", "layer1".."layer4" (int8 NHWC) or
 * "gap" (int8 [B][512]).  *bytes receives the size. */
int dlq_resnet18_stage(dlq_resnet18* m, const char* name, void* dst, size_t cap, size_t* bytes,
                       void* stream);
/* Per-launch kernel timing: with timing on, every forward records one
 * hipEvent on its stream before each kernel launch (tagged with the launch's
 * kernel family below) and one after the last, so launch i lasts
 * elapsed(event i, event i+1).  dlq_resnet18_timing synchronises, fills
 * ms[DLQ_FAM_COUNT] (summed milliseconds) and launches[DLQ_FAM_COUNT] per
 * family, the number of forwards covered, and resets.
 * dlq_resnet18_family_work gives each family's algorithmic MACs and
 * activation bytes (input + output (+ residual), weights excluded) per image
 * and forward, the basis of a roofline's "achieved". */
enum {
  DLQ_FAM_STEM = 0,  /* stem_fused_kernel: quantise + conv1 + BN/ReLU + maxpool */
  DLQ_FAM_L1 = 1,    /* block_l1_kernel: fused layer1 basic blocks             */
  DLQ_FAM_S2DS = 2,  /* conv3x3s2i_kernel: layerX.0 conv1 + fused downsample    */
  DLQ_FAM_WIDE = 3,  /* conv3x3i_kernel: layer2-4 stride-1 3x3 convs            */
  DLQ_FAM_GAP = 4,   /* gap_fc_kernel (int8: GAP + FC) / gap16 (fp8, split)     */
  DLQ_FAM_FC = 5,    /* linear_kernel (FC, when the head is split)              */
  DLQ_FAM_OTHER = 6, /* any unfused fallback launch                             */
  DLQ_FAM_F8 = 7,    /* conv_s8_kernel<..., F8>: every conv of the fp8 path     */
  DLQ_FAM_COUNT = 8
};
int dlq_resnet18_set_timing(dlq_resnet18* m, int on);
int dlq_resnet18_timing(dlq_resnet18* m, double* ms, int* launches, int* forwards);
int dlq_resnet18_family_work(const dlq_resnet18* m, double* macs, double* bytes);
/* Algorithmic MACs per image of the 20 convs and of the FC layer. */
int dlq_resnet18_macs_per_image(const dlq_resnet18* m, double* conv_macs, double* fc_macs);

/* The reference's fp32 forward, op for op (RK/runtime/infer_e2e.cu:259-438:
 * im2col-ordered fmaf GEMM convs, bn_inference, relu, add_inplace, maxpool,
 * gap_global_ref, fc_forward + host bias), on the GPU from the model's fp32
 * tensors (an int8 manifest's weights as q * scale): logits[B][1000] fp32
 * (device, nullable) from x[B][3][224][224] (device).  Bit-identical to the
 * reference's fp32 semantics (pinned by out/step8_logits.bin via the oracle);
 * naive kernels -- model preparation and parity, not the int8 hot path.
 * Keeps "stem_pool", "layer1".."layer4", "gap", "logits" (fp32 NCHW) for
 * dlq_resnet18_stage_f32.  Synchronous. */
int dlq_resnet18_forward_f32(dlq_resnet18* m, const float* x, int B, float* logits, void* stream);
int dlq_resnet18_stage_f32(dlq_resnet18* m, const char* name, void* dst, size_t cap, size_t* bytes, void* stream);
/* Activation-scale calibration (the "quant block" of RK reports/Step1.md:92):
 * dlq_resnet18_forward_f32 over x[B] and every site's scale set to
 * float(max(amax, 1e-8) / qmax) (qmax 127 for int8, 448 for fp8).  Needs a
 * new dlq_resnet18_prepare afterwards.  Synchronous. */
int dlq_resnet18_calibrate(dlq_resnet18* m, const float* x, int B, float qmax, void* stream);

/* ------------------------------------------------------------------------ */
/* MNIST MLP (CUDA/MNIST_on_GPU/v4.cu forward_timed :255-302, v5.cu        */
/* forward_pass_only :127-157): in -> hidden (ReLU) -> out, int8.           */
/* ------------------------------------------------------------------------ */
typedef struct dlq_mlp dlq_mlp;
/* W1[in][hidden], W2[hidden][out] in the reference's [in][out] layout
 * (v4.cu:121-132 computes X[B][in] @ W[in][out]). */
int dlq_mlp_create(int in, int hidden, int out, const float* W1, const float* b1, const float* W2,
                   const float* b2, float s_in, float s_hidden, int max_batch, void* stream,
                   dlq_mlp** m);
void dlq_mlp_destroy(dlq_mlp* m);
int dlq_mlp_forward(dlq_mlp* m, const float* x, int B, float* logits, void* stream);
/* Copy the int8 hidden activations [B][hidden] of the last forward (device
 * to device, async on `stream`); cap = bytes available at dst. */
int dlq_mlp_copy_hidden(const dlq_mlp* m, int B, int8_t* dst, size_t cap, void* stream);

/* ------------------------------------------------------------------------ */
/* The ends of the path: preprocessing and head.    */
/* ------------------------------------------------------------------------ */
/* Resized size of an H x W image: shorter side 256, the other
 * round(long * 256 / short) half-to-even (RK/tools/preprocess_to_bin.py:8-16). */
int dlq_preprocess_size(int H, int W, int* new_h, int* new_w);
/* N u8 RGB images [N][H][W][3] (HWC, as np.array(PIL image)) -> fp32 NCHW
 * [N][3][224][224]: Pillow BILINEAR resize of the shorter side to 256 (its
 * 8-bit fixed-point resampler, bit-exact), centre crop 224, x/255,
 * (x - mean)/std in fp32 (RK/tools/preprocess_to_bin.py:5-33; the input the
 * reference uploads at RK/runtime/infer_e2e.cu:255-256).  Downscale factor
 * at most 7. */
int dlq_preprocess_u8(const uint8_t* img, int N, int H, int W, float* out, void* stream);
/* softmax_1d (RK/kernels/softmax.cu:5-47) on each of N rows of K logits
 * (expf and IEEE division: within (2e-6 + 2e-7 |x - max|) relative of an
 * exact softmax). */
int dlq_softmax_f32(const float* x, int N, int K, float* y, void* stream);
/* Top-1 per row as the launcher prints it (RK/runtime/infer_e2e.cu:436-438):
 * the first index whose logit beats the running best (initially -1e30);
 * idx = -1 if none does.  val may be NULL. */
int dlq_top1_f32(const float* x, int N, int K, int* idx, float* val, void* stream);

/* ------------------------------------------------------------------------ */
/* fp8 (e4m3) variant: BASELINE configs[4] / SURVEY.md §8(f) row 4.  No     */
/* reference code exists for it (the reference is fp32 + this build's int8 */
/* scheme); each entry point below is the e4m3 twin of the int8 one named.  */
/* Values are OCP e4m3fn bytes (uint8): activations at a per-tensor scale   */
/* (amax/448), weights per output channel (max|w|/448).  Requantisation:    */
/* clamp(y, lo, 448), -0 -> +0, round to nearest even (lo = 0 with ReLU,    */
/* -448 without).  Conv products accumulate in fp32 on                      */
/* v_mfma_f32_32x32x64_f8f6f4; GAP and FC are exact (see oracle.c).         */
/* ------------------------------------------------------------------------ */
/* twin of dlq_quantize_weights_s8: scale[o] = max|w|/448 (1 if zero). */
int dlq_quantize_weights_f8(const float* w, int OC, int K, uint8_t* q, float* scale);
/* twin of dlq_quantize_f32_s8 (x 16-B aligned, q 4-B aligned). */
int dlq_quantize_f32_f8(const float* x, size_t n, float inv_s, uint8_t* q, void* stream);
/* twin of dlq_quantize_nchw_to_nhwc_s8. */
int dlq_quantize_nchw_to_nhwc_f8(const float* x, int N, int C, int H, int W, int Cout, float inv_s, uint8_t* y,
                                 void* stream);
/* Packed image: the int8 wide layout (dlq_pack_conv_weights_s8's) for the
 * layer2-4 3x3 convs (stride 1 and the stride-2 conv1s), else the generic
 * one (C % 64 == 0 or the 7x7 C == 4 stem). */
size_t dlq_conv_packed_bytes_f8(const dlq_conv_desc* d);
int dlq_pack_conv_weights_f8(const dlq_conv_desc* d, const uint8_t* q_oihw, int IC, uint8_t* packed);
/* twin of dlq_conv2d_nhwc_s8 (DLQ_OUT_S8 semantics, e4m3 in and out):
 *   y = fmaf(acc, alpha[o], beta[o]) [+ fmaf(dec(res), res_scale, y)], requant. */
int dlq_conv2d_nhwc_f8(const dlq_conv_desc* d, const uint8_t* x, const uint8_t* w_packed, const float* alpha,
                       const float* beta, const uint8_t* residual, float res_scale, int relu, uint8_t* y,
                       void* stream);
/* twin of dlq_conv2d_s2_ds_nhwc_s8: the 3x3/s2 conv (+BN+ReLU, w_packed from
 * dlq_pack_conv_weights_f8) and the block's 1x1/s2 downsample (+BN, w_ds =
 * dlq_pack_downsample_weights_s8 of the e4m3 codes: the packing moves bytes)
 * of one input in one launch.  Each equals its dlq_conv2d_nhwc_f8 call within
 * the conv bound. */
int dlq_conv2d_s2_ds_nhwc_f8(const dlq_conv_desc* d, const uint8_t* x, const uint8_t* w_packed, const float* alpha,
                             const float* beta, const uint8_t* w_ds, const float* alpha_ds, const float* beta_ds,
                             uint8_t* y, uint8_t* y_ds, void* stream);
/* The raw fp32 accumulators of the same conv (twin of DLQ_OUT_S32): acc
 * NHWC [N][OH][OW][OC] fp32 (parity / debugging). */
int dlq_conv2d_nhwc_f8_acc(const dlq_conv_desc* d, const uint8_t* x, const uint8_t* w_packed, float* acc,
                           void* stream);
/* twin of dlq_pack_stem_weights_s8 / dlq_stem_fused_s8 (quantise + conv1 +
 * BN/ReLU + maxpool in one launch; the rows of channels with alpha < 0 get
 * their sign bits flipped).  Equal, within the conv bound, to
 * dlq_quantize_nchw_to_nhwc_f8 + dlq_conv2d_nhwc_f8 (stem) + the maxpool. */
int dlq_pack_stem_weights_f8(const uint8_t* q_oihw, const float* alpha, uint8_t* packed, float* alpha_packed);
int dlq_stem_fused_f8(const float* x, int N, const uint8_t* w_stem, const float* alpha, const float* beta,
                      float inv_s, uint8_t* y, void* stream);
/* twin of dlq_block_l1_nhwc_s8 (the layer1 basic block in one launch;
 * w1, w2 from dlq_pack_conv_weights_f8 for {N, 56, 56, 64, 64, 3, 3, 1, 1,
 * 1, 1}).  Equal, within the conv bound, to two dlq_conv2d_nhwc_f8 calls. */
int dlq_block_l1_nhwc_f8(const uint8_t* x, int N, const uint8_t* w1, const float* alpha1, const float* beta1,
                         const uint8_t* w2, const float* alpha2, const float* beta2, float s_res, uint8_t* y,
                         void* stream);
/* twin of dlq_gap_nhwc_s8: exact sum of the values in units of 2^-9, then
 * requant(float(sum) * k) with k = s_in/HW/s_out * 2^-9.  The int8
 * dlq_maxpool2d_3x3_s2p1_nhwc_s8 applies unchanged to non-negative e4m3. */
int dlq_gap_nhwc_f8(const uint8_t* x, int N, int C, int HW, float k, uint8_t* y, void* stream);
/* twin of dlq_fc_s8: logits[N][O] = fmaf(float(acc), alpha[o], beta[o]), acc
 * exact (fp64); w row-major [O][K] e4m3 (not packed). */
int dlq_linear_f8(const uint8_t* x, int N, int K, const uint8_t* w, int O, const float* alpha, const float* beta,
                  float* y, void* stream);
/* Engine precision (before dlq_resnet18_prepare): DLQ_PREC_INT8 (default)
 * or DLQ_PREC_FP8 (activation scales then calibrated as amax/448). */
#define DLQ_PREC_INT8 0
#define DLQ_PREC_FP8 1
int dlq_resnet18_set_precision(dlq_resnet18* m, int precision);

#ifdef __cplusplus
}
#endif
#endif /* DLQ_H */
