/*
 * oracle.c -- CPU restatement of the yeontachi/DLQ ResNet-18 / MNIST-FC hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker, never the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it.  The shipped path (libdlq.so) never links or calls anything here.
 *
 * Two families of functions:
 *   ora_*_f32  -- the reference's fp32 semantics, op for op.  The reference
 *                 GPU build contracts `acc += a*b` to FMA (nvcc -fmad=true,
 *                 cpp/CMakeLists.txt:7-8 sets no flags), so every GEMM here
 *                 is a k-ordered fmaf chain.  Pinned bit-exactly by the
 *                 reference's own golden vector out/step8_logits.bin
 *                 (tests/test_oracle.py).
 *   ora_*_s8   -- the int8 path.  The reference has NO int8 code (SURVEY.md
 *                 §0.1); the scheme is the build's own and this
 *                 file is its definition.  Integer parts are exact; the fp32
 *                 epilogue is a fixed sequence of IEEE ops (explicit fmaf,
 *                 rintf = round-half-even) that the HIP kernels repeat.
 *
 * Build: oracle/Makefile (gcc -O3 -ffp-contract=off).  Layouts are the
 * reference's: NCHW activations, OIHW weights, per-image im2col rows ordered
 * r = c*kH*kW + kh*kW + kw (kernels/im2col.cu:37-54).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORA_API __attribute__((visibility("default")))

static inline int out_dim(int in, int k, int s, int p) { return (in + 2 * p - k) / s + 1; }

/* ------------------------------------------------------------------ */
/* fp32 reference semantics                                            */
/* ------------------------------------------------------------------ */

/* kernels/im2col.cu:5-58 -- one image; col[r][oh*OW+ow], zero padding. */
ORA_API void ora_im2col_nchw_f32(const float* x, int C, int H, int W, int kH, int kW, int sH,
                                 int sW, int pH, int pW, float* col) {
  const int OH = out_dim(H, kH, sH, pH), OW = out_dim(W, kW, sW, pW);
  const int cs = OH * OW;
  for (int c = 0; c < C; ++c)
    for (int kh = 0; kh < kH; ++kh)
      for (int kw = 0; kw < kW; ++kw) {
        const int r = c * kH * kW + kh * kW + kw;
        for (int oh = 0; oh < OH; ++oh)
          for (int ow = 0; ow < OW; ++ow) {
            const int ih = oh * sH - pH + kh, iw = ow * sW - pW + kw;
            float v = 0.f;
            if (ih >= 0 && iw >= 0 && ih < H && iw < W) v = x[(size_t)c * H * W + ih * W + iw];
            col[(size_t)r * cs + oh * OW + ow] = v;
          }
      }
}

/* kernels/sgemm_tiled.cu:22-45 -- C[M][N] = A[M][K] * B[K][N], row-major.
 * Each output is acc = fmaf(A[m][k], B[k][n], acc) for k = 0..K-1 in order
 * (the contracted form of `acc += As*Bs`, sgemm_tiled.cu:36).  The loop is
 * k-outer/n-inner so it vectorises while keeping every element's k order. */
ORA_API void ora_sgemm_f32(const float* A, const float* B, float* C, int M, int N, int K) {
  for (int m = 0; m < M; ++m) {
    float* c = C + (size_t)m * N;
    for (int n = 0; n < N; ++n) c[n] = 0.f;
    for (int k = 0; k < K; ++k) {
      const float a = A[(size_t)m * K + k];
      const float* b = B + (size_t)k * N;
      for (int n = 0; n < N; ++n) c[n] = fmaf(a, b[n], c[n]);
    }
  }
}

/* kernels/bn_inference.cu:22-27 -- in place, x laid out [C][HW]. */
ORA_API void ora_bn_inference_f32(float* x, const float* g, const float* b, const float* m,
                                  const float* v, float eps, int C, int HW) {
  for (int c = 0; c < C; ++c) {
    const float d = sqrtf(v[c] + eps);
    for (int i = 0; i < HW; ++i) {
      const float y = (x[(size_t)c * HW + i] - m[c]) / d;
      x[(size_t)c * HW + i] = fmaf(g[c], y, b[c]);
    }
  }
}

/* kernels/relu.cu:9 */
ORA_API void ora_relu_f32(float* x, int n) {
  for (int i = 0; i < n; ++i)
    if (x[i] < 0.f) x[i] = 0.f;
}

/* kernels/add.cu:7 */
ORA_API void ora_add_f32(float* y, const float* x, int n) {
  for (int i = 0; i < n; ++i) y[i] += x[i];
}

/* kernels/maxpool2d.cu:14-40 -- 3x3/s2/p1, out-of-bounds taps skipped. */
ORA_API void ora_maxpool_f32(const float* x, int N, int C, int H, int W, float* y) {
  const int OH = out_dim(H, 3, 2, 1), OW = out_dim(W, 3, 2, 1);
  for (int nc = 0; nc < N * C; ++nc)
    for (int oh = 0; oh < OH; ++oh)
      for (int ow = 0; ow < OW; ++ow) {
        float vmax = -FLT_MAX;
        for (int kh = 0; kh < 3; ++kh) {
          const int ih = oh * 2 - 1 + kh;
          if (ih < 0 || ih >= H) continue;
          for (int kw = 0; kw < 3; ++kw) {
            const int iw = ow * 2 - 1 + kw;
            if (iw < 0 || iw >= W) continue;
            const float v = x[(size_t)nc * H * W + ih * W + iw];
            vmax = v > vmax ? v : vmax;
          }
        }
        y[(size_t)nc * OH * OW + oh * OW + ow] = vmax;
      }
}

/* runtime/infer_e2e.cu:37-61 (gap_global_ref; kernels/gap_global.cu has the
 * same order): 256 strided partial sums, then a tree over strides 128..1. */
ORA_API void ora_gap_f32(const float* x, int C, int HW, float* y) {
  float s[256];
  for (int c = 0; c < C; ++c) {
    for (int t = 0; t < 256; ++t) {
      float acc = 0.f;
      for (int i = t; i < HW; i += 256) acc += x[(size_t)c * HW + i];
      s[t] = acc;
    }
    for (int st = 128; st > 0; st >>= 1)
      for (int t = 0; t < st; ++t) s[t] += s[t + st];
    y[c] = s[0] / (float)HW;
  }
}

/* runtime/infer_e2e.cu:206-219 -- GEMM W[O][I] * gap[I] (N=1) then a host
 * fp32 bias add. */
ORA_API void ora_fc_forward_f32(const float* gap, const float* W, const float* B, int O, int I,
                                float* out) {
  ora_sgemm_f32(W, gap, out, O, 1, I);
  for (int o = 0; o < O; ++o) out[o] += B[o];
}

/* runtime/infer_e2e.cu:102-136 -- conv as im2col + GEMM; weights OIHW are
 * already the GEMM A operand [OC][IC*kH*kW] (the repack loop :114-126 is an
 * identity permutation).  One image; `col` is caller scratch of
 * IC*kH*kW*OH*OW floats. */
ORA_API void ora_conv2d_f32(const float* x, int IC, int H, int W, const float* w, int OC, int kH,
                            int kW, int sH, int sW, int pH, int pW, float* col, float* y) {
  const int OH = out_dim(H, kH, sH, pH), OW = out_dim(W, kW, sW, pW);
  ora_im2col_nchw_f32(x, IC, H, W, kH, kW, sH, sW, pH, pW, col);
  ora_sgemm_f32(w, col, y, OC, OH * OW, IC * kH * kW);
}

/* CUDA/MNIST_on_GPU/v3.c:125-134 + :168-174 + :161-165 -- one dense layer
 * X[B][I] * W[I][O] (+bias, optional ReLU), plain mul-then-add order. */
ORA_API void ora_mlp_layer_f32(const float* X, const float* Wt, const float* bias, int B, int I,
                               int O, int relu, float* Y) {
  for (int b = 0; b < B; ++b)
    for (int o = 0; o < O; ++o) {
      float acc = 0.f;
      for (int i = 0; i < I; ++i) {
        const float p = X[(size_t)b * I + i] * Wt[(size_t)i * O + o];
        acc = acc + p;
      }
      acc = acc + bias[o];
      if (relu) acc = fmaxf(0.f, acc);
      Y[(size_t)b * O + o] = acc;
    }
}

/* ------------------------------------------------------------------ */
/* int8 path (build-defined)                              */
/* ------------------------------------------------------------------ */

static inline int8_t sat_rne(float y) {
  float q = rintf(y);
  q = q < -127.f ? -127.f : q;
  q = q > 127.f ? 127.f : q;
  return (int8_t)(int)q;
}

/* Symmetric per-output-channel weight quantisation over K contiguous
 * values: s[o] = max|w|/127 (1 if the row is all zero), q = sat(rne(w/s)). */
ORA_API void ora_quantize_weights_s8(const float* w, int OC, int K, int8_t* q, float* scale) {
  for (int o = 0; o < OC; ++o) {
    float mx = 0.f;
    for (int k = 0; k < K; ++k) {
      const float a = fabsf(w[(size_t)o * K + k]);
      mx = a > mx ? a : mx;
    }
    const float s = mx > 0.f ? mx / 127.f : 1.f;
    scale[o] = s;
    for (int k = 0; k < K; ++k) q[(size_t)o * K + k] = sat_rne(w[(size_t)o * K + k] / s);
  }
}

/* Fold dequant, BN (kernels/bn_inference.cu:22-27) and the output requant
 * scale into one affine per output channel, in units of the output int8 grid:
 *   t = g/sqrtf(v+eps);  inv_y = 1/s_y;
 *   alpha = ((s_x*s_w)*t)*inv_y;  beta = (b - m*t)*inv_y. */
ORA_API void ora_fold_bn(float s_x, const float* s_w, const float* g, const float* b,
                         const float* m, const float* v, float eps, float s_y, int OC,
                         float* alpha, float* beta) {
  const float inv_y = 1.0f / s_y;
  for (int o = 0; o < OC; ++o) {
    const float t = g[o] / sqrtf(v[o] + eps);
    const float sxw = s_x * s_w[o];
    const float a = sxw * t;
    alpha[o] = a * inv_y;
    const float mt = m[o] * t;
    const float bb = b[o] - mt;
    beta[o] = bb * inv_y;
  }
}

/* Residual scale in output-grid units: s_r * (1/s_y). */
ORA_API float ora_res_scale(float s_r, float s_y) { return s_r * (1.0f / s_y); }

/* fp32 -> int8 with one per-tensor scale: q = sat(rne(x * inv_s)). */
ORA_API void ora_quantize_f32_s8(const float* x, size_t n, float inv_s, int8_t* q) {
  for (size_t i = 0; i < n; ++i) q[i] = sat_rne(x[i] * inv_s);
}

/* im2col.cu:37-54 on int8 (one image). */
ORA_API void ora_im2col_nchw_s8(const int8_t* x, int C, int H, int W, int kH, int kW, int sH,
                                int sW, int pH, int pW, int8_t* col) {
  const int OH = out_dim(H, kH, sH, pH), OW = out_dim(W, kW, sW, pW);
  const int cs = OH * OW;
  for (int c = 0; c < C; ++c)
    for (int kh = 0; kh < kH; ++kh)
      for (int kw = 0; kw < kW; ++kw) {
        const int r = c * kH * kW + kh * kW + kw;
        for (int oh = 0; oh < OH; ++oh)
          for (int ow = 0; ow < OW; ++ow) {
            const int ih = oh * sH - pH + kh, iw = ow * sW - pW + kw;
            int8_t v = 0;
            if (ih >= 0 && iw >= 0 && ih < H && iw < W) v = x[(size_t)c * H * W + ih * W + iw];
            col[(size_t)r * cs + oh * OW + ow] = v;
          }
      }
}

/* sgemm_tiled.cu's C = A*B on int8 operands with int32 accumulation. */
ORA_API void ora_gemm_s8s8s32(const int8_t* A, const int8_t* B, int32_t* C, int M, int N, int K) {
  for (int m = 0; m < M; ++m) {
    int32_t* c = C + (size_t)m * N;
    for (int n = 0; n < N; ++n) c[n] = 0;
    for (int k = 0; k < K; ++k) {
      const int32_t a = A[(size_t)m * K + k];
      if (a == 0) continue;
      const int8_t* b = B + (size_t)k * N;
      for (int n = 0; n < N; ++n) c[n] += a * (int32_t)b[n];
    }
  }
}

/* conv2d_nchw_im2col_gemm (infer_e2e.cu:102-136) on int8: int32
 * accumulators acc[N][OC][OH][OW]; w is [OC][IC*kH*kW] int8. */
ORA_API int ora_conv2d_nchw_s8_acc(const int8_t* x, int N, int IC, int H, int W, const int8_t* w,
                                   int OC, int kH, int kW, int sH, int sW, int pH, int pW,
                                   int32_t* acc) {
  const int OH = out_dim(H, kH, sH, pH), OW = out_dim(W, kW, sW, pW);
  const size_t K = (size_t)IC * kH * kW;
  int8_t* col = (int8_t*)malloc(K * OH * OW);
  if (!col) return 1;
  for (int n = 0; n < N; ++n) {
    ora_im2col_nchw_s8(x + (size_t)n * IC * H * W, IC, H, W, kH, kW, sH, sW, pH, pW, col);
    ora_gemm_s8s8s32(w, col, acc + (size_t)n * OC * OH * OW, OC, OH * OW, (int)K);
  }
  free(col);
  return 0;
}

/* Fused epilogue (replaces bn_inference + add_inplace + relu_forward,
 * infer_e2e.cu:168-200) on NCHW accumulators, alpha/beta/r_s already in
 * output-grid units (ora_fold_bn, ora_res_scale):
 *   y = fmaf(float(acc), alpha[c], beta[c])
 *   y = fmaf(float(res), r_s, y)            if res != NULL
 *   q = rne(clamp(y, relu ? 0 : -127, 127))                              */
ORA_API void ora_epilogue_s8(const int32_t* acc, int N, int OC, int HW, const float* alpha,
                             const float* beta, const int8_t* res, float r_s, int relu,
                             int8_t* out) {
  const float lo = relu ? 0.f : -127.f;
  for (int n = 0; n < N; ++n)
    for (int c = 0; c < OC; ++c)
      for (int i = 0; i < HW; ++i) {
        const size_t idx = ((size_t)n * OC + c) * HW + i;
        float y = fmaf((float)acc[idx], alpha[c], beta[c]);
        if (res) y = fmaf((float)res[idx], r_s, y);
        y = y < lo ? lo : y;
        y = y > 127.f ? 127.f : y;
        out[idx] = (int8_t)(int)rintf(y);
      }
}

/* add_inplace (RK/kernels/add.cu:7) + relu in the int8 domain:
 * y = clamp(rne(fmaf(r, r_s, a * a_s)), relu ? 0 : -127, 127). */
ORA_API void ora_add_requant_s8(const int8_t* a, const int8_t* r, size_t n, float a_s, float r_s, int relu,
                                int8_t* out) {
  const float lo = relu ? 0.f : -127.f;
  for (size_t i = 0; i < n; ++i) {
    float y = fmaf((float)r[i], r_s, (float)a[i] * a_s);
    y = y < lo ? lo : y;
    y = y > 127.f ? 127.f : y;
    out[i] = (int8_t)(int)rintf(y);
  }
}

/* fp32 epilogue (FC logits / dequant): y = fmaf(float(acc), alpha, beta). */
ORA_API void ora_epilogue_f32(const int32_t* acc, int N, int OC, int HW, const float* alpha,
                              const float* beta, int relu, float* out) {
  for (int n = 0; n < N; ++n)
    for (int c = 0; c < OC; ++c)
      for (int i = 0; i < HW; ++i) {
        const size_t idx = ((size_t)n * OC + c) * HW + i;
        float y = fmaf((float)acc[idx], alpha[c], beta[c]);
        if (relu) y = y > 0.f ? y : 0.f;
        out[idx] = y;
      }
}

/* maxpool2d.cu:14-40 on int8 (exact: requant is monotone). */
ORA_API void ora_maxpool_s8(const int8_t* x, int N, int C, int H, int W, int8_t* y) {
  const int OH = out_dim(H, 3, 2, 1), OW = out_dim(W, 3, 2, 1);
  for (int nc = 0; nc < N * C; ++nc)
    for (int oh = 0; oh < OH; ++oh)
      for (int ow = 0; ow < OW; ++ow) {
        int vmax = -128;
        for (int kh = 0; kh < 3; ++kh) {
          const int ih = oh * 2 - 1 + kh;
          if (ih < 0 || ih >= H) continue;
          for (int kw = 0; kw < 3; ++kw) {
            const int iw = ow * 2 - 1 + kw;
            if (iw < 0 || iw >= W) continue;
            const int v = x[(size_t)nc * H * W + ih * W + iw];
            vmax = v > vmax ? v : vmax;
          }
        }
        y[(size_t)nc * OH * OW + oh * OW + ow] = (int8_t)vmax;
      }
}

/* GAP (infer_e2e.cu:37-61) on int8: exact int32 channel sum, then one
 * requant q = sat(rne(float(sum) * k)) with k = s_in/(HW*s_out) from the
 * host.  sums (optional) receives the int32 sums [N][C]. */
ORA_API void ora_gap_s8(const int8_t* x, int N, int C, int HW, float k, int32_t* sums,
                        int8_t* y) {
  for (int nc = 0; nc < N * C; ++nc) {
    int32_t s = 0;
    for (int i = 0; i < HW; ++i) s += x[(size_t)nc * HW + i];
    if (sums) sums[nc] = s;
    y[nc] = sat_rne((float)s * k);
  }
}

/* FC (infer_e2e.cu:206-219) on int8, batched: acc[n][o] = sum_k x[n][k]*W[o][k],
 * logits = fmaf(float(acc), alpha[o], beta[o]).  accs (optional) gets int32. */
ORA_API void ora_fc_s8(const int8_t* x, int N, int I, const int8_t* W, int O, const float* alpha,
                       const float* beta, int32_t* accs, float* out) {
  for (int n = 0; n < N; ++n)
    for (int o = 0; o < O; ++o) {
      int32_t s = 0;
      for (int k = 0; k < I; ++k) s += (int32_t)x[(size_t)n * I + k] * W[(size_t)o * I + k];
      if (accs) accs[(size_t)n * O + o] = s;
      out[(size_t)n * O + o] = fmaf((float)s, alpha[o], beta[o]);
    }
}

/* MNIST FC layer on int8 (v4.cu:121-132 / v5.cu:131-150 semantics, W stored
 * [in][out] as in the reference): acc[b][o] = sum_i x[b][i]*Wt[i][o]. */
ORA_API void ora_mlp_layer_s8_acc(const int8_t* x, const int8_t* Wt, int B, int I, int O,
                                  int32_t* acc) {
  for (int b = 0; b < B; ++b) {
    int32_t* c = acc + (size_t)b * O;
    for (int o = 0; o < O; ++o) c[o] = 0;
    for (int i = 0; i < I; ++i) {
      const int32_t a = x[(size_t)b * I + i];
      for (int o = 0; o < O; ++o) c[o] += a * (int32_t)Wt[(size_t)i * O + o];
    }
  }
}

/* ------------------------------------------------------------------ */
/* fp8 path (BASELINE configs[4]; build-defined, */
/* DESIGN.md §3b).  No reference code exists for it.                    */
/* ------------------------------------------------------------------ */
/* Values are OCP e4m3fn bytes: sign, 4 exponent bits (bias 7), 3 mantissa
 * bits, max 448, 0x7F/0xFF NaN (never produced: every encode clamps to
 * +-448 first).  Every e4m3 value is an integer multiple of 2^-9 (the
 * smallest subnormal), so a code's "units" (value * 512) are an exact
 * integer <= 229376, products of units are exact int64 multiples of 2^-18
 * and every sum here is exact: the oracle's conv / FC accumulators are the
 * exact real sums, returned as doubles (exact: |sum| * 2^18 < 2^53). */

static int32_t f8_units_tab[256];
static int f8_tab_ready = 0;

static void f8_init(void) {
  if (f8_tab_ready) return;
  for (int c = 0; c < 256; ++c) {
    const int e = (c >> 3) & 15, m = c & 7;
    /* subnormal: m * 2^-9 -> m units; normal: (8+m) * 2^(e-7-3) -> (8+m) << (e-1) units */
    int32_t u = e == 0 ? m : (8 + m) << (e - 1);
    if ((c & 0x7f) == 0x7f) u = 0; /* NaN: never produced or consumed */
    f8_units_tab[c] = (c & 0x80) ? -u : u;
  }
  f8_tab_ready = 1;
}

ORA_API float ora_f8_decode(uint8_t c) {
  f8_init();
  float v = ldexpf((float)f8_units_tab[c], -9);
  if (c == 0x80) v = -0.0f;
  return v;
}

/* Round-to-nearest-even e4m3 encode of y, |y| <= 448 (callers clamp).  The
 * sign bit is y's (a negative value that rounds to zero gives 0x80). */
static uint8_t f8_encode(float y) {
  const uint8_t sgn = signbit(y) ? 0x80 : 0;
  const float a = fabsf(y);
  uint8_t code;
  if (a < 0x1p-6f) {
    code = (uint8_t)(int)rintf(a * 512.f); /* subnormal grid 2^-9; 8 = smallest normal */
  } else {
    int e;
    frexpf(a, &e);                /* a = f * 2^e, f in [0.5, 1) -> unbiased exponent e-1 */
    const int E = e - 1;          /* -6 .. 8 */
    int r = (int)rintf(ldexpf(a, 3 - E)); /* mantissa with hidden bit, 8 .. 16 */
    int eb = E + 7;
    if (r == 16) { r = 8; ++eb; }
    code = (uint8_t)((eb << 3) | (r - 8));
  }
  return code | sgn;
}

/* clamp(y, lo, 448), -0 -> +0 (y + 0.0f), encode: the requantisation of the
 * fp8 scheme, repeated op for op by device_common.h enc4_f8. */
static inline uint8_t f8_requant(float y, float lo) {
  y = y < lo ? lo : y;
  y = y > 448.f ? 448.f : y;
  return f8_encode(y + 0.0f);
}

ORA_API void ora_encode_f8(const float* y, size_t n, uint8_t* q) {
  for (size_t i = 0; i < n; ++i) q[i] = f8_encode(y[i]);
}

ORA_API void ora_decode_f8(const uint8_t* q, size_t n, float* y) {
  for (size_t i = 0; i < n; ++i) y[i] = ora_f8_decode(q[i]);
}

/* fp32 -> e4m3 activation quantisation: q = requant(x * inv_s, -448). */
ORA_API void ora_quantize_f32_f8(const float* x, size_t n, float inv_s, uint8_t* q) {
  for (size_t i = 0; i < n; ++i) q[i] = f8_requant(x[i] * inv_s, -448.f);
}

/* Per-output-channel e4m3 weights: s[o] = max|w|/448 (1 if all zero),
 * q = requant(w / s, -448). */
ORA_API void ora_quantize_weights_f8(const float* w, int OC, int K, uint8_t* q, float* scale) {
  for (int o = 0; o < OC; ++o) {
    float mx = 0.f;
    for (int k = 0; k < K; ++k) {
      const float a = fabsf(w[(size_t)o * K + k]);
      mx = a > mx ? a : mx;
    }
    const float s = mx > 0.f ? mx / 448.f : 1.f;
    scale[o] = s;
    for (int k = 0; k < K; ++k) q[(size_t)o * K + k] = f8_requant(w[(size_t)o * K + k] / s, -448.f);
  }
}

/* Exact accumulators of an e4m3 conv (NCHW codes, OIHW codes), as doubles. */
ORA_API int ora_conv2d_nchw_f8_acc(const uint8_t* x, int N, int IC, int H, int W, const uint8_t* w, int OC,
                                   int kH, int kW, int sH, int sW, int pH, int pW, double* acc) {
  f8_init();
  const int OH = out_dim(H, kH, sH, pH), OW = out_dim(W, kW, sW, pW);
  const size_t K = (size_t)IC * kH * kW, P = (size_t)OH * OW;
  int8_t* col = (int8_t*)malloc(K * P);
  int32_t* cu = (int32_t*)malloc(K * P * sizeof(int32_t));
  int64_t* row = (int64_t*)malloc(P * sizeof(int64_t));
  if (!col || !cu || !row) {
    free(col); free(cu); free(row);
    return 1;
  }
  for (int n = 0; n < N; ++n) {
    /* zero padding = code 0x00 = +0 */
    ora_im2col_nchw_s8((const int8_t*)x + (size_t)n * IC * H * W, IC, H, W, kH, kW, sH, sW, pH, pW, col);
    for (size_t i = 0; i < K * P; ++i) cu[i] = f8_units_tab[(uint8_t)col[i]];
    for (int o = 0; o < OC; ++o) {
      memset(row, 0, P * sizeof(int64_t));
      for (size_t k = 0; k < K; ++k) {
        const int64_t a = f8_units_tab[w[(size_t)o * K + k]];
        if (!a) continue;
        const int32_t* c = cu + k * P;
        for (size_t p = 0; p < P; ++p) row[p] += a * c[p];
      }
      double* d = acc + ((size_t)n * OC + o) * P;
      for (size_t p = 0; p < P; ++p) d[p] = ldexp((double)row[p], -18);
    }
  }
  free(col); free(cu); free(row);
  return 0;
}

/* fp8 fused epilogue on NCHW accumulators (alpha/beta/r_s in output-grid
 * units, as ora_epilogue_s8):
 *   y = fmaf(float(acc), alpha[c], beta[c]);  y = fmaf(dec(res), r_s, y)
 *   q = requant(y, relu ? 0 : -448)                                       */
ORA_API void ora_epilogue_f8(const double* acc, int N, int OC, int HW, const float* alpha, const float* beta,
                             const uint8_t* res, float r_s, int relu, uint8_t* out) {
  const float lo = relu ? 0.f : -448.f;
  for (int n = 0; n < N; ++n)
    for (int c = 0; c < OC; ++c)
      for (int i = 0; i < HW; ++i) {
        const size_t idx = ((size_t)n * OC + c) * HW + i;
        float y = fmaf((float)acc[idx], alpha[c], beta[c]);
        if (res) y = fmaf(ora_f8_decode(res[idx]), r_s, y);
        out[idx] = f8_requant(y, lo);
      }
}

/* GAP on e4m3: exact unit sums S (int32), y = requant(float(S) * k, -448)
 * with k = gap_k(s_in, hw, s_out) * 2^-9 (the units' scale). */
ORA_API void ora_gap_f8(const uint8_t* x, int N, int C, int HW, float k, int32_t* sums, uint8_t* y) {
  f8_init();
  for (int nc = 0; nc < N * C; ++nc) {
    int32_t s = 0;
    for (int i = 0; i < HW; ++i) s += f8_units_tab[x[(size_t)nc * HW + i]];
    if (sums) sums[nc] = s;
    y[nc] = f8_requant((float)s * k, -448.f);
  }
}

/* FC on e4m3: exact acc, logits = fmaf(float(acc), alpha[o], beta[o]). */
ORA_API void ora_fc_f8(const uint8_t* x, int N, int I, const uint8_t* W, int O, const float* alpha,
                       const float* beta, double* accs, float* out) {
  f8_init();
  for (int n = 0; n < N; ++n)
    for (int o = 0; o < O; ++o) {
      int64_t s = 0;
      for (int k = 0; k < I; ++k)
        s += (int64_t)f8_units_tab[x[(size_t)n * I + k]] * f8_units_tab[W[(size_t)o * I + k]];
      const double a = ldexp((double)s, -18);
      if (accs) accs[(size_t)n * O + o] = a;
      out[(size_t)n * O + o] = fmaf((float)a, alpha[o], beta[o]);
    }
}
