// mlp.cpp -- int8 MNIST MLP forward behind dlq_mlp_* (include/dlq.h).
//
// Mirrors the forward half of CUDA/MNIST_on_GPU/v4.cu forward_timed
// (:255-302: matmul_a_b_kernel -> bias_forward_kernel -> relu_forward_kernel
// -> matmul_a_b_kernel -> bias_forward_kernel) and v5.cu forward_pass_only
// (:127-157, cublasSgemm + bias_add_kernel + relu_kernel).  The softmax
// (v4.cu:182-200) and the training half (backward, SGD) are out of scope.
// The whole forward is ONE launch (head.hip mlp_fused_kernel: quantise, fc1 +
// bias + ReLU + requant, fc2 + bias, the hidden layer kept in LDS); the
// reference issues five kernels and a cudaDeviceSynchronize per op
// (v4.cu:260-265).  Shapes whose rows + hidden layer do not fit the fused
// kernel's 64 KiB of LDS (wide inputs or hidden layers, e.g. in 16K or
// hidden 8192) run the same integer sums and IEEE epilogues as three
// launches: quantize_rows -> linear (+ ReLU, requant) -> linear (fp32 out).
#include <cstring>
#include <vector>

#include "../../include/dlq.h"
#include "dlq_internal.h"

using namespace dlq;

struct dlq_mlp {
  int in = 0, hidden = 0, out = 0, kp = 0, max_batch = 0;
  float s_in = 1.f, s_hidden = 1.f;
  int8_t* w1 = nullptr;  // packed [OCp(hidden)][kp] (fused: its fragment-major image)
  int8_t* w2 = nullptr;  // packed [OCp(out)][hidden] (fused: its fragment-major image)
  float *a1 = nullptr, *b1 = nullptr, *a2 = nullptr, *b2 = nullptr;
  bool fused = true;      // mlp_fused_fits(kp, hidden, out)
  int8_t* xq = nullptr;  // [max_batch][kp], the three-launch path only
  int8_t* hq = nullptr;  // [max_batch][hidden]
  std::vector<void*> allocs;
};

namespace {

int up(dlq_mlp* m, void** dst, const void* src, size_t bytes) {
  hipError_t e = hipMalloc(dst, bytes ? bytes : 16);
  if (e != hipSuccess) return hip_fail(e, "hipMalloc");
  m->allocs.push_back(*dst);
  if (src && bytes) {
    e = hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpy");
  }
  return DLQ_OK;
}

// Reference layout W[in][out] (v4.cu:121-132) -> per-output-channel int8
// rows, packed [OCp][kp]; alpha = s_x * s_w[o], beta = bias[o] -- for an int8
// output (s_y > 0) both in output-grid units: alpha = (s_x*s_w[o])*(1/s_y),
// beta = bias[o]*(1/s_y) (the convention of dlq_fold_bn).
// The fused kernel's fragment-major image of a generic packed [OCp][kp]
// image (head.hip mlp_frag): fragment (k-step k, tile t) at (k * T + t) *
// 1024, lane l = 32 lh + r its A-fragment bytes -- row t * 32 + r, k-bytes
// 32 k + 16 lh .. +15, read where the generic image keeps them (the
// addressing of the kernels that read it, mlp_wfrag's before): one
// contiguous KiB per wave-wide fragment load.
std::vector<int8_t> mlp_fragment_image(const std::vector<int8_t>& g, int OCp, int kp) {
  const int T = OCp / 32, nk = kp / 32;
  const size_t ws = (size_t)(OCp / 64) * 64 * 64;
  std::vector<int8_t> f(g.size());
  for (int k = 0; k < nk; ++k)
    for (int t = 0; t < T; ++t)
      for (int l = 0; l < 64; ++l) {
        const int oc = t * 32 + (l & 31), lh = l >> 5, ol = oc & 63, sw = (ol >> 2) & 3;
        const size_t src = (size_t)(k >> 1) * ws + ((size_t)(oc >> 6) * 64 + ol) * 64 + ((((2 * k + lh) & 3) ^ sw) << 4);
        std::memcpy(&f[((size_t)k * T + t) * 1024 + l * 16], &g[src], 16);
      }
  return f;
}

int prep_layer(dlq_mlp* m, const float* Wt, const float* bias, int in, int out, int kp, float s_x,
               float s_y, int8_t** dw, float** da, float** db, bool frag) {
  std::vector<float> w((size_t)out * in);
  for (int i = 0; i < in; ++i)
    for (int o = 0; o < out; ++o) w[(size_t)o * in + i] = Wt[(size_t)i * out + o];
  std::vector<int8_t> q(w.size());
  std::vector<float> sw(out);
  quantize_weights(w.data(), out, in, q.data(), sw.data());
  std::vector<int8_t> packed(packed_bytes(out, kp, 1, 1));
  pack_conv_weights(q.data(), out, in, 1, 1, kp, packed.data());
  const int op = packed_oc(out);
  if (frag) packed = mlp_fragment_image(packed, op, kp);
  std::vector<float> a(op, 0.f), b(op, 0.f);
  const float inv_y = s_y > 0.f ? 1.0f / s_y : 1.0f;
  for (int o = 0; o < out; ++o) {
    const float sa = s_x * sw[o];
    a[o] = s_y > 0.f ? sa * inv_y : sa;
    b[o] = s_y > 0.f ? bias[o] * inv_y : bias[o];
  }
  int rc;
  if ((rc = up(m, (void**)dw, packed.data(), packed.size())) || (rc = up(m, (void**)da, a.data(), op * 4)) ||
      (rc = up(m, (void**)db, b.data(), op * 4)))
    return rc;
  return DLQ_OK;
}

}  // namespace

extern "C" {

int dlq_mlp_create(int in, int hidden, int out, const float* W1, const float* b1, const float* W2,
                   const float* b2, float s_in, float s_hidden, int max_batch, void* stream,
                   dlq_mlp** res) {
  (void)stream;
  if (!res || !W1 || !b1 || !W2 || !b2 || in <= 0 || hidden <= 0 || out <= 0 || max_batch <= 0)
    return fail(DLQ_ERR_ARG, "mlp_create: bad args");
  if (hidden % 64) return fail(DLQ_ERR_ARG, "mlp_create: hidden must be a multiple of 64");
  if (!(s_in > 0.f) || !(s_hidden > 0.f)) return fail(DLQ_ERR_ARG, "mlp_create: scales must be > 0");
  auto* m = new dlq_mlp();
  m->in = in; m->hidden = hidden; m->out = out; m->kp = (in + 63) / 64 * 64;
  m->max_batch = max_batch; m->s_in = s_in; m->s_hidden = s_hidden;
  m->fused = mlp_fused_fits(m->kp, hidden, out);
  int rc;
  if ((rc = prep_layer(m, W1, b1, in, hidden, m->kp, s_in, s_hidden, &m->w1, &m->a1, &m->b1, m->fused)) ||
      (rc = prep_layer(m, W2, b2, hidden, out, hidden, s_hidden, 0.f, &m->w2, &m->a2, &m->b2, m->fused)) ||
      (!m->fused && (rc = up(m, (void**)&m->xq, nullptr, (size_t)max_batch * m->kp))) ||
      (rc = up(m, (void**)&m->hq, nullptr, (size_t)max_batch * hidden))) {
    dlq_mlp_destroy(m);
    return rc;
  }
  *res = m;
  return DLQ_OK;
}

void dlq_mlp_destroy(dlq_mlp* m) {
  if (!m) return;
  for (void* p : m->allocs) (void)hipFree(p);
  delete m;
}

int dlq_mlp_forward(dlq_mlp* m, const float* x, int B, float* logits, void* stream) {
  if (!m) return fail(DLQ_ERR_ARG, "mlp_forward: null model");
  if (B < 0 || B > m->max_batch) return fail(DLQ_ERR_ARG, "mlp_forward: batch exceeds max_batch");
  if (B == 0) return DLQ_OK;
  if (!x || !logits) return fail(DLQ_ERR_ARG, "mlp_forward: null argument");
  const hipStream_t s = (hipStream_t)stream;
  if (m->fused) {
    const hipError_t e = launch_mlp_fused(x, B, m->in, m->kp, 1.0f / m->s_in, m->w1, m->hidden, m->a1, m->b1, m->w2,
                                          m->out, m->a2, m->b2, m->hq, logits, s);
    return e == hipSuccess ? DLQ_OK : hip_fail(e, "mlp_forward");
  }
  hipError_t e = launch_quantize_rows(x, B, m->in, m->kp, 1.0f / m->s_in, m->xq, s);
  if (e == hipSuccess) e = launch_linear(m->xq, B, m->kp, m->w1, m->hidden, m->a1, m->b1, 1, 0, m->hq, s);
  if (e == hipSuccess) e = launch_linear(m->hq, B, m->hidden, m->w2, m->out, m->a2, m->b2, 0, 1, logits, s);
  return e == hipSuccess ? DLQ_OK : hip_fail(e, "mlp_forward (three-launch path)");
}

int dlq_mlp_copy_hidden(const dlq_mlp* m, int B, int8_t* dst, size_t cap, void* stream) {
  if (!m || !dst || B < 0 || B > m->max_batch) return fail(DLQ_ERR_ARG, "mlp_copy_hidden: bad args");
  const size_t bytes = (size_t)B * m->hidden;
  if (cap < bytes) return fail(DLQ_ERR_ARG, "mlp_copy_hidden: destination too small");
  hipError_t e = hipMemcpyAsync(dst, m->hq, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream);
  return e == hipSuccess ? DLQ_OK : hip_fail(e, "mlp_copy_hidden");
}

}  // extern "C"
