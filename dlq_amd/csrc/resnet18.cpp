// resnet18.cpp -- the ResNet-18 int8 engine behind dlq_resnet18_* (include/dlq.h).
//
// Host-side mirror of the reference launcher
// CUDA/resnet18-kernel-lab/cpp/fp32/runtime/infer_e2e.cu:
//   conv2d_nhwc_s8      <- conv2d_nchw_im2col_gemm  (:102-136) + bn_launch (:83-97)
//   basic_block_forward <- basic_block_forward       (:139-203, BlockParams :139-152)
//   fc_forward          <- fc_forward                (:206-219)
//   forward()           <- main()'s stage sequence   (:253-433)
// Differences that are the point of the rebuild: weights are quantised,
// BN-folded and uploaded ONCE (prepare), not re-read from disk and copied
// H2D per call (:262, :304-334, :128); no cudaMalloc/cudaFree or host sync
// inside forward (the reference frees temporaries per layer and syncs at
// :280, :292, :423); the batch dimension is honoured; BN, ReLU, residual add
// and requantisation run in the conv kernel's epilogue.
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <sys/stat.h>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/dlq.h"
#include "dlq_internal.h"

using namespace dlq;

namespace {

struct ConvLayer {
  std::string site;     // activation-scale site of this conv's OUTPUT, e.g. "layer1.0.conv1"
  std::string wname;    // state_dict weight name
  std::string bn;       // state_dict BN prefix
  std::string in_site;  // scale site of the INPUT activation
  int IC = 0, OC = 0, k = 0, s = 1, p = 0, Cstore = 0;
  int H = 0;            // input height = width
  int8_t* w = nullptr;  // packed weights (device)
  int8_t* wf = nullptr; // downsample convs: the fused stride-2 kernel's layout (dlq_pack_downsample_weights_s8)
  float* alpha = nullptr;
  float* beta = nullptr;
};

struct Block {
  std::string name;
  int ic, oc, stride;
  bool down;
  int c1, c2, ds;  // indices into convs (ds = -1 if identity)
};

}  // namespace

struct QTensor {  // pre-quantised weight (int8 manifest): per-output-channel int8 + scales
  std::vector<int8_t> q;
  std::vector<float> scale;
};

struct dlq_resnet18 {
  std::map<std::string, std::vector<float>> tensors;
  std::map<std::string, QTensor> qtensors;
  std::map<std::string, float> scales;
  std::vector<ConvLayer> convs;
  std::vector<Block> blocks;
  int stem = -1;
  int8_t* stem_w = nullptr;       // fused-stem weight image (dlq_pack_stem_weights_s8)
  float* stem_alpha = nullptr;    // |alpha| of conv1 for the fused stem
  // FC
  int8_t* fc_w = nullptr;
  float* fc_alpha = nullptr;
  float* fc_beta = nullptr;
  // workspace
  int max_batch = 0;
  int8_t* buf[4] = {};        // block activations, each B*56*56*64 bytes
  int8_t* gq = nullptr;       // [B][512]
  std::vector<void*> allocs;
  bool prepared = false;
  // stage pointers of the last forward
  std::map<std::string, std::pair<const int8_t*, size_t>> stage;
  int last_B = 0;
  // optional per-stage copies (parity dumps; infer_e2e.cu maybe_save :243-248)
  bool keep = false;
  std::map<std::string, int8_t*> keepbuf;
  // optional per-launch timing: one hipEvent before every kernel launch
  // (tagged with the launch's kernel family, DLQ_FAM_*) and one after the
  // last; launch i's duration = elapsed(ev[i], ev[i+1]) on the forward's stream.
  bool timing = false;
  std::vector<hipEvent_t> ev;
  std::vector<int> ev_tag;  // family of the launch that follows, -1 = end of forward
  size_t ev_used = 0;
  // half-batch split: a second stream runs the second half of the batch in
  // its own half of every workspace buffer, so the two halves' launches
  // interleave and fill each other's tail waves
  hipStream_t s2 = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  // DLQ_PREC_INT8 / DLQ_PREC_FP8 (e4m3 activations + per-channel e4m3
  // weights; generic packed layout in ConvLayer::w, fc_w row-major codes)
  int prec = DLQ_PREC_INT8;
  // hipGraph of one whole forward (every launch of forward_pass), captured on
  // a private stream the first time a (x, B, logits) triple is seen and
  // replayed on the caller's stream afterwards: one submission per forward
  // instead of ~16 kernel launches.  Kernel arguments (weights, workspace,
  // x, logits) are baked in, so prepare / precision changes drop it.
  hipStream_t gs = nullptr;
  hipGraphExec_t gexec = nullptr;
  unsigned g_gen = 0;  // g_knob_gen at capture
  const float* g_x = nullptr;
  float* g_logits = nullptr;
  int g_B = 0;
  // stage outputs of the last reference-semantics fp32 forward
  // (dlq_resnet18_forward_f32): fp32 NCHW device buffers owned here
  std::map<std::string, std::pair<float*, size_t>> stage_f32;
};

namespace {

const int kBlocks[8][4] = {  // in, out, stride, downsample (infer_e2e.cu:336-407)
    {64, 64, 1, 0},  {64, 64, 1, 0},  {64, 128, 2, 1},  {128, 128, 1, 0},
    {128, 256, 2, 1}, {256, 256, 1, 0}, {256, 512, 2, 1}, {512, 512, 1, 0}};
const char* kBlockNames[8] = {"layer1.0", "layer1.1", "layer2.0", "layer2.1",
                              "layer3.0", "layer3.1", "layer4.0", "layer4.1"};

void build_topology(dlq_resnet18* m) {
  m->convs.clear();
  m->blocks.clear();
  ConvLayer st;
  st.site = "conv1"; st.wname = "conv1.weight"; st.bn = "bn1"; st.in_site = "input";
  st.IC = 3; st.OC = 64; st.k = 7; st.s = 2; st.p = 3; st.Cstore = kStemC; st.H = 224;
  m->convs.push_back(st);
  m->stem = 0;
  std::string prev = "conv1";
  int H = 56;
  for (int b = 0; b < 8; ++b) {
    const std::string n = kBlockNames[b];
    Block blk{n, kBlocks[b][0], kBlocks[b][1], kBlocks[b][2], kBlocks[b][3] != 0, 0, 0, -1};
    ConvLayer c1;
    c1.site = n + ".conv1"; c1.wname = n + ".conv1.weight"; c1.bn = n + ".bn1"; c1.in_site = prev;
    c1.IC = blk.ic; c1.OC = blk.oc; c1.k = 3; c1.s = blk.stride; c1.p = 1; c1.Cstore = blk.ic; c1.H = H;
    blk.c1 = (int)m->convs.size();
    m->convs.push_back(c1);
    if (blk.down) {
      ConvLayer d;
      d.site = n + ".downsample"; d.wname = n + ".downsample.0.weight"; d.bn = n + ".downsample.1";
      d.in_site = prev;
      d.IC = blk.ic; d.OC = blk.oc; d.k = 1; d.s = blk.stride; d.p = 0; d.Cstore = blk.ic; d.H = H;
      blk.ds = (int)m->convs.size();
      m->convs.push_back(d);
    }
    ConvLayer c2;
    c2.site = n + ".conv2"; c2.wname = n + ".conv2.weight"; c2.bn = n + ".bn2"; c2.in_site = c1.site;
    H /= blk.stride;
    c2.IC = blk.oc; c2.OC = blk.oc; c2.k = 3; c2.s = 1; c2.p = 1; c2.Cstore = blk.oc; c2.H = H;
    blk.c2 = (int)m->convs.size();
    m->convs.push_back(c2);
    m->blocks.push_back(blk);
    prev = c2.site;
  }
}

std::vector<std::string> required_tensors(const dlq_resnet18* m) {
  std::vector<std::string> r;
  for (const auto& c : m->convs) {
    r.push_back(c.wname);
    for (const char* s : {".weight", ".bias", ".running_mean", ".running_var"}) r.push_back(c.bn + s);
  }
  r.push_back("fc.weight");
  r.push_back("fc.bias");
  return r;
}

size_t expected_numel(const dlq_resnet18* m, const std::string& name) {
  for (const auto& c : m->convs) {
    if (name == c.wname) return (size_t)c.OC * c.IC * c.k * c.k;
    if (name.compare(0, c.bn.size() + 1, c.bn + ".") == 0) {
      const std::string rest = name.substr(c.bn.size() + 1);
      if (rest == "weight" || rest == "bias" || rest == "running_mean" || rest == "running_var")
        return (size_t)c.OC;
    }
  }
  if (name == "fc.weight") return 1000 * 512;
  if (name == "fc.bias") return 1000;
  return 0;
}

template <typename T>
int dev_alloc(dlq_resnet18* m, T** p, size_t bytes) {
  void* q = nullptr;
  hipError_t e = hipMalloc(&q, bytes ? bytes : 16);
  if (e != hipSuccess) return hip_fail(e, "hipMalloc");
  m->allocs.push_back(q);
  *p = (T*)q;
  return DLQ_OK;
}

void drop_graph(dlq_resnet18* m) {
  if (m->gexec) (void)hipGraphExecDestroy(m->gexec);
  m->gexec = nullptr;
  m->g_x = nullptr;
  m->g_logits = nullptr;
  m->g_B = 0;
}

void free_all(dlq_resnet18* m) {
  drop_graph(m);
  for (void* p : m->allocs) (void)hipFree(p);
  m->allocs.clear();
  for (auto& c : m->convs) { c.w = nullptr; c.wf = nullptr; c.alpha = nullptr; c.beta = nullptr; }
  m->fc_w = nullptr; m->fc_alpha = m->fc_beta = nullptr;
  m->gq = m->stem_w = nullptr;
  m->stem_alpha = nullptr;
  for (auto& b : m->buf) b = nullptr;
  m->keepbuf.clear();
  m->prepared = false;
}

float inv_scale(float s) { return 1.0f / s; }

// Knob "head_split" (DLQ_HEAD_SPLIT=1, dlq_set_knob): GAP and FC as two
// launches (gap16_kernel + linear_kernel) instead of the fused gap_fc_kernel.
bool head_split() { return g_knob_head_split.load(std::memory_order_relaxed) == 1; }

// Knob "ds_split" (DLQ_DS_SPLIT): 0 = default on, -1 = off.  A downsampling
// block's 1x1/s2 downsample is computed by its conv2 launch (conv3x3i DSR;
// layer2.0 and layer3.0) and its stride-2 conv1 runs alone, instead of the
// downsample fused into the stride-2 launch (conv3x3s2i DS, stored and read
// back as conv2's residual; layer4.0 always, or every block with -1).
// 1 / 2: only layer3.0 (14x14 output) / only layer2.0 (28x28) (A/B of the two)
bool ds_split(int OH) {
  const int k = g_knob_ds_split.load(std::memory_order_relaxed);
  return k == 0 || (k == 1 && OH == 14) || (k == 2 && OH == 28) || k > 2;
}

// Knob "prefetch" (DLQ_PREFETCH): 0 = default on, -1 = off.  Each wide /
// stride-2 conv launch's last stage reads the next launch's first weight
// stages (Prefetch, device_common.h prefetch_next).
bool prefetch_on() { return g_knob_prefetch.load(std::memory_order_relaxed) >= 0; }

// Knob "gap_epi" (DLQ_GAP_EPI): 0 = default on, -1 = off.  The last conv
// (layer4.1 conv2) pools its own output (conv3x3i GAP) and the head is the
// FC alone (linear512_f32_kernel), instead of the fused gap_fc_kernel.
bool gap_epi_on() { return g_knob_gap_epi.load(std::memory_order_relaxed) >= 0; }

// conv2d_nchw_im2col_gemm + bn_launch (+ add_inplace + relu_forward) of the
// reference, as one implicit-GEMM launch with the epilogue fused.
int conv2d_nhwc_s8(const dlq_resnet18* m, const ConvLayer& c, const int8_t* x, int N, int H, int W,
                   const int8_t* residual, float res_scale, bool relu, int8_t* y, hipStream_t s,
                   int* OH, int* OW, const Prefetch* pf = nullptr, int8_t* gap_y = nullptr, float gap_k = 0.f) {
  dlq_conv_desc d{N, H, W, c.Cstore, c.OC, c.k, c.k, c.s, c.s, c.p, c.p};
  *OH = out_dim(H, c.k, c.s, c.p);
  *OW = out_dim(W, c.k, c.s, c.p);
  // alpha/beta are already in this conv's output-grid units (prepare); the
  // residual's scale is converted the same way.
  const float r_s = residual ? dlq::res_scale(res_scale, m->scales.at(c.site)) : 0.f;
  return conv2d_nhwc_s8_pf(&d, x, c.w, c.alpha, c.beta, residual, r_s, relu ? 1 : 0, DLQ_OUT_S8, y, s, pf, gap_y,
                           gap_k);
}

// The first weight stages a launch of conv `c` (input H x H) streams: the
// wide image's first four 32-channel slices of every 128-channel block (and
// of the fused downsample's image), or none for other layouts.
Prefetch conv_prefetch(const ConvLayer& c, int H, const ConvLayer* ds = nullptr) {
  Prefetch pf{};
  if (!(c.k == 3 && wide_layout(c.Cstore, c.OC, H, H, 3, 3, c.s, c.s, 1, 1))) return pf;
  const int NS = c.Cstore / 32, ns = NS < 4 ? NS : 4, nb = packed_oc(c.OC) / 128;
  pf.p[0] = c.w;
  pf.n[0] = nb;
  pf.stride[0] = NS * 128 * 304;
  pf.len[0] = ns * 128 * 304;
  if (ds && ds->wf) {
    pf.p[1] = ds->wf;
    pf.n[1] = nb;
    pf.stride[1] = NS * 128 * 48;
    pf.len[1] = ns * 128 * 48;
  }
  return pf;
}

int mark(dlq_resnet18* m, hipStream_t s, int family) {
  if (!m->timing) return DLQ_OK;
  if (m->ev_used == m->ev.size()) {
    if (m->ev.size() >= 32 * 4096) return fail(DLQ_ERR_STATE, "timing: event pool full; call dlq_resnet18_timing");
    hipEvent_t e;
    hipError_t he = hipEventCreate(&e);
    if (he != hipSuccess) return hip_fail(he, "hipEventCreate");
    m->ev.push_back(e);
    m->ev_tag.push_back(-1);
  }
  m->ev_tag[m->ev_used] = family;
  hipError_t he = hipEventRecord(m->ev[m->ev_used++], s);
  return he == hipSuccess ? DLQ_OK : hip_fail(he, "hipEventRecord");
}

// Kernel family of a conv launch (for the per-launch timing).
int conv_family(const ConvLayer& c, int H) {
  if (c.k == 3 && c.s == 1 && conv3x3w_shape(c.Cstore, c.OC, H, H, 3, 3, 1, 1, 1, 1) &&
      wide_layout(c.Cstore, c.OC, H, H, 3, 3, 1, 1, 1, 1))
    return DLQ_FAM_WIDE;
  if (c.k == 3 && c.s == 1 && c.Cstore == 64 && H == 56) return DLQ_FAM_L1;
  return DLQ_FAM_OTHER;
}

// The layer1 blocks (64 -> 64 channels at 56x56, identity skip) run as one
// fused launch each (block_l1.hip).
bool fused_l1_block(const dlq_resnet18* m, const Block& b, int H, int W) {
  if (b.down) return false;
  const ConvLayer& c1 = m->convs[b.c1];
  const ConvLayer& c2 = m->convs[b.c2];
  return c1.k == 3 && c1.s == 1 && c1.p == 1 && c2.k == 3 && c2.s == 1 && c2.p == 1 &&
         block_l1_shape(c1.Cstore, c1.OC, H, W) && block_l1_shape(c2.Cstore, c2.OC, H, W) &&
         !wide_layout(c1.Cstore, c1.OC, H, W, 3, 3, 1, 1, 1, 1);
}

// The first weights the first launch of block `b` (input H x H) reads: the
// fused layer1 block's two weight images, or its first conv's stages.
Prefetch block_prefetch(const dlq_resnet18* m, const Block& b, int H) {
  if (fused_l1_block(m, b, H, H)) {
    Prefetch pf{};
    const int len = (int)packed_bytes(64, 64, 3, 3);
    pf.p[0] = m->convs[b.c1].w;
    pf.p[1] = m->convs[b.c2].w;
    pf.n[0] = pf.n[1] = 1;
    pf.len[0] = pf.len[1] = len;
    return pf;
  }
  return conv_prefetch(m->convs[b.c1], H, b.down ? &m->convs[b.ds] : nullptr);
}

// basic_block_forward (infer_e2e.cu:156-203): conv-bn-relu, conv-bn,
// identity | 1x1 downsample-bn, add, relu -- three launches at most.
int basic_block_forward(dlq_resnet18* m, const Block& b, const int8_t* in, int N, int H,
                        int W, int8_t* h, int8_t* dsb, int8_t* out, hipStream_t s, int* OH,
                        int* OW, const Prefetch* next = nullptr, int8_t* gap_y = nullptr, float gap_k = 0.f) {
  int h1, w1, h2, w2;
  const ConvLayer& c1 = m->convs[b.c1];
  const int8_t* skip = in;
  float s_skip = m->scales.at(c1.in_site);
  int rc;
  if (fused_l1_block(m, b, H, W)) {
    // both convs, the identity add and the ReLUs in one launch; the
    // intermediate never leaves the CU (block_l1.hip)
    const ConvLayer& c2 = m->convs[b.c2];
    if ((rc = mark(m, s, DLQ_FAM_L1))) return rc;
    const float r_s = dlq::res_scale(s_skip, m->scales.at(c2.site));
    hipError_t e = launch_block_l1(in, N, c1.w, c1.alpha, c1.beta, c2.w, c2.alpha, c2.beta, r_s, out, s, false,
                                   prefetch_on() ? next : nullptr);
    if (e != hipSuccess) return hip_fail(e, "block_l1 launch");
    *OH = H;
    *OW = W;
    return DLQ_OK;
  }
  const ConvLayer* c2w = &m->convs[b.c2];
  if (b.down && m->convs[b.ds].wf && ds_split(H / 2) && conv3x3s2_shape(c1.Cstore, c1.OC, H, W, 3, 3, 2, 2, 1, 1) &&
      wide_layout(c1.Cstore, c1.OC, H, W, 3, 3, 2, 2, 1, 1) &&
      conv3x3w_shape(c2w->Cstore, c2w->OC, H / 2, W / 2, 3, 3, 1, 1, 1, 1) && H / 2 != 7 && c2w->Cstore == c1.OC &&
      m->convs[b.ds].OC == c1.OC && 2 * c1.Cstore == c1.OC) {
    // conv1 (3x3/s2) alone, then conv2 with the 1x1/s2 downsample computed
    // and requantised in its epilogue as the residual (conv3x3i DSR): the
    // downsample's output never goes to memory
    const ConvLayer& ds = m->convs[b.ds];
    const ConvLayer& c2 = *c2w;
    dlq_conv_desc d{N, H, W, c1.Cstore, c1.OC, 3, 3, 2, 2, 1, 1};
    if ((rc = mark(m, s, DLQ_FAM_S2DS))) return rc;
    h1 = out_dim(H, 3, 2, 1);
    w1 = out_dim(W, 3, 2, 1);
    const Prefetch pf2 = conv_prefetch(c2, h1);
    rc = conv2d_nhwc_s8_pf(&d, in, c1.w, c1.alpha, c1.beta, nullptr, 0.f, 1, DLQ_OUT_S8, h, s,
                           prefetch_on() ? &pf2 : nullptr);
    if (rc) return rc;
    if ((rc = mark(m, s, conv_family(c2, h1)))) return rc;
    dlq_conv_desc d2{N, h1, w1, c2.Cstore, c2.OC, 3, 3, 1, 1, 1, 1};
    ConvArgs a;
    const float r_s = dlq::res_scale(m->scales.at(ds.site), m->scales.at(c2.site));
    if ((rc = conv_args_checked(&d2, h, c2.w, c2.alpha, c2.beta, nullptr, r_s, 1, DLQ_OUT_S8, out, a))) return rc;
    a.ds_x = in;
    a.ds_w = ds.wf;
    a.ds_alpha = ds.alpha;
    a.ds_beta = ds.beta;
    a.ds_C = c1.Cstore;
    if (next && prefetch_on()) a.pf = *next;
    if (a.P) {
      hipError_t e = launch_conv3x3i_dsr(a, s);
      if (e != hipSuccess) return hip_fail(e, "conv2 + downsample residual launch");
    }
    *OH = h1;
    *OW = w1;
    return DLQ_OK;
  }
  if (b.down && m->convs[b.ds].wf && conv3x3s2_shape(c1.Cstore, c1.OC, H, W, 3, 3, 2, 2, 1, 1) &&
      wide_layout(c1.Cstore, c1.OC, H, W, 3, 3, 2, 2, 1, 1)) {
    // conv1 (3x3/s2) and the 1x1/s2 downsample in one launch
    const ConvLayer& ds = m->convs[b.ds];
    dlq_conv_desc d{N, H, W, c1.Cstore, c1.OC, 3, 3, 2, 2, 1, 1};
    if ((rc = mark(m, s, DLQ_FAM_S2DS))) return rc;
    const Prefetch pf2 = conv_prefetch(m->convs[b.c2], out_dim(H, 3, 2, 1));
    rc = conv2d_s2_ds_nhwc_s8_pf(&d, in, c1.w, c1.alpha, c1.beta, ds.wf, ds.alpha, ds.beta, h, dsb, s,
                                 prefetch_on() ? &pf2 : nullptr);
    if (rc) return rc;
    h1 = out_dim(H, 3, 2, 1);
    w1 = out_dim(W, 3, 2, 1);
    skip = dsb;
    s_skip = m->scales.at(ds.site);
  } else {
    if ((rc = mark(m, s, conv_family(c1, H)))) return rc;
    const Prefetch pf2 = conv_prefetch(m->convs[b.c2], out_dim(H, 3, c1.s, 1));
    rc = conv2d_nhwc_s8(m, c1, in, N, H, W, nullptr, 0.f, true, h, s, &h1, &w1,
                        !b.down && prefetch_on() ? &pf2 : nullptr);
    if (rc) return rc;
    if (b.down) {
      int hd, wd;
      if ((rc = mark(m, s, DLQ_FAM_OTHER))) return rc;
      rc = conv2d_nhwc_s8(m, m->convs[b.ds], in, N, H, W, nullptr, 0.f, false, dsb, s, &hd, &wd);
      if (rc) return rc;
      if (hd != h1 || wd != w1) return fail(DLQ_ERR_STATE, "downsample shape mismatch");
      skip = dsb;
      s_skip = m->scales.at(m->convs[b.ds].site);
    }
  }
  if ((rc = mark(m, s, conv_family(m->convs[b.c2], h1)))) return rc;
  rc = conv2d_nhwc_s8(m, m->convs[b.c2], h, N, h1, w1, skip, s_skip, true, out, s, &h2, &w2,
                      prefetch_on() ? next : nullptr, gap_y, gap_k);
  *OH = h2;
  *OW = w2;
  return rc;
}

// Record a stage output; with keep_stages on, snapshot it (the block ring
// buffers are reused by later layers).
int record_stage(dlq_resnet18* m, const char* name, const int8_t* p, size_t bytes, hipStream_t s) {
  auto it = m->keepbuf.find(name);
  if (m->keep && it != m->keepbuf.end()) {
    hipError_t e = hipMemcpyAsync(it->second, p, bytes, hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return hip_fail(e, "stage snapshot");
    p = it->second;
  }
  m->stage[name] = {p, bytes};
  return DLQ_OK;
}

// Output channels of a weight tensor (conv or fc), 0 if `name` is not one.
int weight_oc(const dlq_resnet18* m, const std::string& name) {
  for (const auto& c : m->convs)
    if (name == c.wname) return c.OC;
  return name == "fc.weight" ? 1000 : 0;
}

// The int8 weights + per-channel scales of a weight tensor: as set
// pre-quantised (int8 manifest), or quantised now from fp32 (same function,
// so both routes give the same bytes).
void weights_s8(const dlq_resnet18* m, const std::string& name, int OC, int K, std::vector<int8_t>& q,
                std::vector<float>& sw) {
  auto it = m->qtensors.find(name);
  if (it != m->qtensors.end()) {
    q = it->second.q;
    sw = it->second.scale;
    return;
  }
  q.resize((size_t)OC * K);
  sw.resize(OC);
  quantize_weights(m->tensors.at(name).data(), OC, K, q.data(), sw.data());
}

// fp32 values of a weight tensor for the fp8 path: the fp32 tensor, or the
// int8 manifest's q * scale[o] when only that was given.
std::vector<float> weights_f32(const dlq_resnet18* m, const std::string& name, int OC, int K) {
  auto t = m->tensors.find(name);
  if (t != m->tensors.end()) return t->second;
  const QTensor& qt = m->qtensors.at(name);
  std::vector<float> w((size_t)OC * K);
  for (int o = 0; o < OC; ++o)
    for (int k = 0; k < K; ++k) w[(size_t)o * K + k] = (float)qt.q[(size_t)o * K + k] * qt.scale[o];
  return w;
}

int check_ready(const dlq_resnet18* m) {
  for (const auto& n : required_tensors(m))
    if (!m->tensors.count(n) && !m->qtensors.count(n)) return fail(DLQ_ERR_STATE, "missing tensor: " + n);
  std::vector<std::string> sites = {"input", "gap"};
  for (const auto& c : m->convs) sites.push_back(c.site);
  for (const auto& s : sites)
    if (!m->scales.count(s)) return fail(DLQ_ERR_STATE, "missing activation scale: " + s);
  return DLQ_OK;
}

}  // namespace

namespace {
// Whole file -> bytes (load_bin_f32, RK/include/utils.hpp:48-60, for any element type).
int read_file(const std::string& path, std::vector<char>& out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return fail(DLQ_ERR_IO, "open fail: " + path);
  f.seekg(0, std::ios::end);
  const size_t bytes = (size_t)f.tellg();
  f.seekg(0);
  out.resize(bytes);
  if (bytes) f.read(out.data(), (std::streamsize)bytes);
  if (!f) return fail(DLQ_ERR_IO, "read fail: " + path);
  return DLQ_OK;
}

int write_file(const std::string& path, const void* p, size_t bytes) {
  std::ofstream f(path, std::ios::binary);
  if (!f) return fail(DLQ_ERR_IO, "open fail: " + path);
  if (bytes) f.write((const char*)p, (std::streamsize)bytes);
  if (!f) return fail(DLQ_ERR_IO, "write fail: " + path);
  return DLQ_OK;
}

// manifest.json's "dtype" (the reference writes "fp32", export_resnet18.py:68-72);
// "fp32" when there is no manifest.json (a bare directory of .bin files).
std::string manifest_dtype(const std::string& dir) {
  std::ifstream f(dir + "/manifest.json");
  if (!f) return "fp32";
  const std::string s((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  const size_t k = s.find("\"dtype\"");
  if (k == std::string::npos) return "fp32";
  const size_t a = s.find('"', s.find(':', k) + 1), b = a == std::string::npos ? a : s.find('"', a + 1);
  return (a == std::string::npos || b == std::string::npos) ? "fp32" : s.substr(a + 1, b - a - 1);
}

std::vector<int> tensor_shape(const dlq_resnet18* m, const std::string& name) {
  for (const auto& c : m->convs)
    if (name == c.wname) return {c.OC, c.IC, c.k, c.k};
  if (name == "fc.weight") return {1000, 512};
  return {(int)expected_numel(m, name)};
}
}  // namespace

extern "C" {

int dlq_resnet18_create(dlq_resnet18** out) {
  if (!out) return fail(DLQ_ERR_ARG, "resnet18_create: null out");
  auto* m = new dlq_resnet18();
  build_topology(m);
  *out = m;
  return DLQ_OK;
}

void dlq_resnet18_destroy(dlq_resnet18* m) {
  if (m && m->s2) {
    (void)hipStreamSynchronize(m->s2);
    (void)hipStreamDestroy(m->s2);
    (void)hipEventDestroy(m->fork);
    (void)hipEventDestroy(m->join);
    m->s2 = nullptr;
  }
  if (!m) return;
  for (hipEvent_t e : m->ev) (void)hipEventDestroy(e);
  if (m->gexec) (void)hipDeviceSynchronize();  // a replay may still be in flight
  free_all(m);
  for (auto& kv : m->stage_f32) (void)hipFree(kv.second.first);
  if (m->gs) (void)hipStreamDestroy(m->gs);
  delete m;
}

int dlq_resnet18_set_tensor(dlq_resnet18* m, const char* name, const float* data, size_t n) {
  if (!m || !name || !data) return fail(DLQ_ERR_ARG, "set_tensor: null argument");
  const size_t want = expected_numel(m, name);
  if (!want) return fail(DLQ_ERR_ARG, std::string("set_tensor: unknown tensor ") + name);
  if (n != want)
    return fail(DLQ_ERR_ARG, std::string("set_tensor: ") + name + " has " + std::to_string(n) +
                                 " elements, expected " + std::to_string(want));
  m->tensors[name].assign(data, data + n);
  m->qtensors.erase(name);
  m->prepared = false;
  return DLQ_OK;
}

int dlq_resnet18_set_tensor_s8(dlq_resnet18* m, const char* name, const int8_t* q, size_t n, const float* scale,
                               size_t n_scale) {
  if (!m || !name || !q || !scale) return fail(DLQ_ERR_ARG, "set_tensor_s8: null argument");
  const int oc = weight_oc(m, name);
  if (!oc) return fail(DLQ_ERR_ARG, std::string("set_tensor_s8: not a conv / fc weight: ") + name);
  if (n != expected_numel(m, name) || n_scale != (size_t)oc)
    return fail(DLQ_ERR_ARG, std::string("set_tensor_s8: ") + name + ": wrong element or scale count");
  for (size_t i = 0; i < n; ++i)
    if (q[i] == -128) return fail(DLQ_ERR_ARG, std::string("set_tensor_s8: ") + name + ": -128 (range is +-127)");
  for (size_t o = 0; o < n_scale; ++o)
    if (!(scale[o] > 0.f) || !std::isfinite(scale[o]))
      return fail(DLQ_ERR_ARG, std::string("set_tensor_s8: ") + name + ": scales must be finite and > 0");
  QTensor& t = m->qtensors[name];
  t.q.assign(q, q + n);
  t.scale.assign(scale, scale + n_scale);
  m->tensors.erase(name);
  m->prepared = false;
  return DLQ_OK;
}

int dlq_resnet18_set_scale(dlq_resnet18* m, const char* name, float scale) {
  if (!m || !name) return fail(DLQ_ERR_ARG, "set_scale: null argument");
  if (!(scale > 0.f) || !std::isfinite(scale)) return fail(DLQ_ERR_ARG, "set_scale: scale must be finite and > 0");
  m->scales[name] = scale;
  m->prepared = false;
  return DLQ_OK;
}

// load_bin_f32 (utils.hpp:48-60) without the exit(): <dir>/<name>.bin.

int dlq_resnet18_load_manifest(dlq_resnet18* m, const char* dir) {
  if (!m || !dir) return fail(DLQ_ERR_ARG, "load_manifest: null argument");
  const std::string dtype = manifest_dtype(dir);
  if (dtype != "fp32" && dtype != "int8") return fail(DLQ_ERR_IO, "load_manifest: unsupported dtype " + dtype);
  for (const auto& n : required_tensors(m)) {
    const std::string path = std::string(dir) + "/" + n + ".bin";
    std::vector<char> raw;
    int rc = read_file(path, raw);
    if (rc) return rc;
    if (dtype == "int8" && weight_oc(m, n)) {  // int8 weights + <name>.scale.bin (fp32 per output channel)
      std::vector<char> sc;
      if ((rc = read_file(std::string(dir) + "/" + n + ".scale.bin", sc))) return rc;
      if (sc.size() % 4) return fail(DLQ_ERR_IO, "size not float-aligned: " + n + ".scale.bin");
      rc = dlq_resnet18_set_tensor_s8(m, n.c_str(), (const int8_t*)raw.data(), raw.size(), (const float*)sc.data(),
                                      sc.size() / 4);
    } else {
      if (raw.size() % 4) return fail(DLQ_ERR_IO, "size not float-aligned: " + path);
      std::vector<float> v(raw.size() / 4);
      if (!raw.empty()) std::memcpy(v.data(), raw.data(), raw.size());
      rc = dlq_resnet18_set_tensor(m, n.c_str(), v.data(), v.size());
    }
    if (rc) return rc;
  }
  return DLQ_OK;
}

int dlq_resnet18_save_manifest(const dlq_resnet18* m, const char* dir, int int8) {
  if (!m || !dir) return fail(DLQ_ERR_ARG, "save_manifest: null argument");
  for (const auto& n : required_tensors(m)) {
    const bool w = weight_oc(m, n) != 0;
    if (!m->tensors.count(n) && !(w && m->qtensors.count(n)))
      return fail(DLQ_ERR_STATE, "save_manifest: missing tensor " + n);
    if (!int8 && !m->tensors.count(n))
      return fail(DLQ_ERR_STATE, "save_manifest: " + n + " is only held as int8; save it with int8 = 1");
  }
  if (mkdir(dir, 0755) != 0 && errno != EEXIST) return fail(DLQ_ERR_IO, std::string("mkdir fail: ") + dir);
  std::ostringstream js;
  js << "{\n  \"model\": \"resnet18\",\n  \"dtype\": \"" << (int8 ? "int8" : "fp32")
     << "\",\n  \"layout\": \"NCHW\",\n  \"version\": 1,\n"
     << "  \"preprocess\": {\"resize\": 256, \"center_crop\": 224, \"mean\": [0.485, 0.456, 0.406], "
        "\"std\": [0.229, 0.224, 0.225]},\n  \"tensors\": {";
  bool first = true;
  for (const auto& n : required_tensors(m)) {
    const int oc = weight_oc(m, n);
    const std::vector<int> shape = tensor_shape(m, n);
    int rc;
    std::string kind, layout, extra;
    if (oc && shape.size() == 4) kind = "conv_weight", layout = "OIHW";
    else if (oc) kind = "fc_weight", layout = "OI";
    else if (n.find("running_") != std::string::npos) kind = "bn_buffer", layout = "O";
    else if (n == "fc.bias") kind = "fc_bias", layout = "O";
    else kind = "bn_param", layout = "O";
    if (int8 && oc) {
      const int K = (int)(expected_numel(m, n) / oc);
      std::vector<int8_t> q;
      std::vector<float> sw;
      weights_s8(m, n, oc, K, q, sw);
      if ((rc = write_file(std::string(dir) + "/" + n + ".bin", q.data(), q.size())) ||
          (rc = write_file(std::string(dir) + "/" + n + ".scale.bin", sw.data(), sw.size() * 4)))
        return rc;
      extra = ", \"dtype\": \"int8\", \"quant\": \"symmetric_per_out_channel\", \"scale_path\": \"" + n +
              ".scale.bin\"";
    } else {
      const std::vector<float>& v = m->tensors.at(n);
      if ((rc = write_file(std::string(dir) + "/" + n + ".bin", v.data(), v.size() * 4))) return rc;
    }
    js << (first ? "\n" : ",\n") << "    \"" << n << "\": {\"shape\": [";
    for (size_t i = 0; i < shape.size(); ++i) js << (i ? ", " : "") << shape[i];
    js << "], \"layout\": \"" << layout << "\", \"kind\": \"" << kind << "\", \"path\": \"" << n << ".bin\"" << extra
       << "}";
    first = false;
  }
  js << "\n  }\n}\n";
  const std::string j = js.str();
  int rc = write_file(std::string(dir) + "/manifest.json", j.data(), j.size());
  // the activation scales travel with the weights: the launcher reads
  // <dir>/scales.txt when --scales is not given
  if (!rc && !m->scales.empty()) rc = dlq_resnet18_save_scales(m, (std::string(dir) + "/scales.txt").c_str());
  return rc;
}

int dlq_resnet18_save_scales(const dlq_resnet18* m, const char* path) {
  if (!m || !path) return fail(DLQ_ERR_ARG, "save_scales: null argument");
  std::ostringstream o;
  o << "# activation scales (site scale), dlq_resnet18_load_scales format\n";
  o.precision(9);
  for (const auto& kv : m->scales) o << kv.first << " " << kv.second << "\n";
  const std::string t = o.str();
  return write_file(path, t.data(), t.size());
}

int dlq_resnet18_load_scales(dlq_resnet18* m, const char* path) {
  if (!m || !path) return fail(DLQ_ERR_ARG, "load_scales: null argument");
  std::ifstream f(path);
  if (!f) return fail(DLQ_ERR_IO, std::string("open fail: ") + path);
  std::string line;
  while (std::getline(f, line)) {
    if (line.empty() || line[0] == '#') continue;
    std::istringstream ss(line);
    std::string site;
    float s;
    if (!(ss >> site >> s)) return fail(DLQ_ERR_IO, "bad scale line: " + line);
    int rc = dlq_resnet18_set_scale(m, site.c_str(), s);
    if (rc) return rc;
  }
  return DLQ_OK;
}

}  // extern "C"

namespace {
template <typename T>
int upload(dlq_resnet18* m, T** dst, const void* src, size_t bytes) {
  int rc = dev_alloc(m, dst, bytes);
  if (rc) return rc;
  hipError_t e = hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice);
  return e == hipSuccess ? DLQ_OK : hip_fail(e, "weight upload");
}

// fp8 prepare: e4m3 per-channel weights in the generic packed layout, BN
// folded exactly as the int8 path (fold_bn with the e4m3 weight scales),
// FC row-major.
int prepare_f8(dlq_resnet18* m, int max_batch) {
  int rc;
  for (auto& c : m->convs) {
    const int K = c.IC * c.k * c.k, ocp = packed_oc(c.OC);
    const std::vector<float> w = weights_f32(m, c.wname, c.OC, K);
    std::vector<uint8_t> q((size_t)c.OC * K);
    std::vector<float> sw(c.OC);
    quantize_weights_f8(w.data(), c.OC, K, q.data(), sw.data());
    std::vector<uint8_t> packed(packed_bytes_f8(c.Cstore, c.OC, c.H, c.H, c.k, c.k, c.s, c.s, c.p, c.p));
    pack_conv_weights_f8(c.Cstore, c.OC, c.H, c.H, c.k, c.k, c.s, c.s, c.p, c.p, q.data(), c.IC, packed.data());
    std::vector<float> alpha(ocp, 0.f), beta(ocp, 0.f);
    fold_bn(m->scales.at(c.in_site), sw.data(), m->tensors.at(c.bn + ".weight").data(),
            m->tensors.at(c.bn + ".bias").data(), m->tensors.at(c.bn + ".running_mean").data(),
            m->tensors.at(c.bn + ".running_var").data(), 1e-5f, m->scales.at(c.site), c.OC, alpha.data(),
            beta.data());
    if ((rc = upload(m, &c.w, packed.data(), packed.size())) || (rc = upload(m, &c.alpha, alpha.data(), ocp * 4)) ||
        (rc = upload(m, &c.beta, beta.data(), ocp * 4)))
      return rc;
    if (c.k == 1 && c.s == 2 && c.Cstore % 32 == 0) {  // the downsample's image for the fused s2 launch
      std::vector<int8_t> fp(downsample_packed_bytes(c.OC, c.Cstore));
      downsample_pack((const int8_t*)q.data(), c.OC, c.IC, c.Cstore, fp.data());
      if ((rc = upload(m, &c.wf, fp.data(), fp.size()))) return rc;
    }
    if (&c == &m->convs[m->stem]) {  // the fused stem's image (sign bits of alpha < 0 rows flipped)
      std::vector<uint8_t> sp(stem_packed_bytes());
      std::vector<float> sa(64);
      pack_stem_weights_f8(q.data(), alpha.data(), sp.data(), sa.data());
      if ((rc = upload(m, &m->stem_w, sp.data(), sp.size())) || (rc = upload(m, &m->stem_alpha, sa.data(), 64 * 4)))
        return rc;
    }
  }
  {
    const int O = 1000, I = 512;
    const std::vector<float> w = weights_f32(m, "fc.weight", O, I);
    std::vector<uint8_t> q((size_t)O * I);
    std::vector<float> sw(O), alpha(O), beta(O);
    quantize_weights_f8(w.data(), O, I, q.data(), sw.data());
    const float sg = m->scales.at("gap");
    const std::vector<float>& bias = m->tensors.at("fc.bias");
    for (int o = 0; o < O; ++o) {
      alpha[o] = sg * sw[o];
      beta[o] = bias[o];
    }
    if ((rc = upload(m, &m->fc_w, q.data(), q.size())) || (rc = upload(m, &m->fc_alpha, alpha.data(), O * 4)) ||
        (rc = upload(m, &m->fc_beta, beta.data(), O * 4)))
      return rc;
  }
  const size_t B = (size_t)max_batch;
  if ((rc = dev_alloc(m, &m->gq, B * 512))) return rc;
  for (auto& b : m->buf)
    if ((rc = dev_alloc(m, &b, B * 56 * 56 * 64))) return rc;
  if (m->keep) {
    const std::pair<const char*, size_t> kb[] = {{"stem_pool", 56 * 56 * 64}, {"layer1", 56 * 56 * 64},
                                                 {"layer2", 28 * 28 * 128}, {"layer3", 14 * 14 * 256},
                                                 {"layer4", 7 * 7 * 512}};
    for (const auto& k : kb) {
      int8_t* p = nullptr;
      if ((rc = dev_alloc(m, &p, B * k.second))) return rc;
      m->keepbuf[k.first] = p;
    }
  }
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return hip_fail(e, "prepare sync");
  m->max_batch = max_batch;
  m->prepared = true;
  return DLQ_OK;
}
}  // namespace

extern "C" {

int dlq_resnet18_set_precision(dlq_resnet18* m, int precision) {
  if (!m || (precision != DLQ_PREC_INT8 && precision != DLQ_PREC_FP8))
    return fail(DLQ_ERR_ARG, "set_precision: DLQ_PREC_INT8 or DLQ_PREC_FP8");
  if (m->prec != precision) {
    m->prec = precision;
    m->prepared = false;  // weights and workspace must be prepared again
  }
  return DLQ_OK;
}

int dlq_resnet18_prepare(dlq_resnet18* m, int max_batch, void* stream) {
  if (!m || max_batch <= 0) return fail(DLQ_ERR_ARG, "prepare: bad args");
  if (max_batch > kMaxBatch) return fail(DLQ_ERR_ARG, "prepare: max_batch above kMaxBatch (int32 activation offsets)");
  int rc = check_ready(m);
  if (rc) return rc;
  free_all(m);
  hipStream_t s = (hipStream_t)stream;
  if (m->prec == DLQ_PREC_FP8) return prepare_f8(m, max_batch);
  // Weights: quantise per output channel, fold BN, pack, upload once.
  for (auto& c : m->convs) {
    const int K = c.IC * c.k * c.k;
    const int ocp = packed_oc(c.OC);
    std::vector<int8_t> q;
    std::vector<float> sw;
    weights_s8(m, c.wname, c.OC, K, q, sw);
    const size_t pb = packed_bytes_for(c.Cstore, c.OC, c.H, c.H, c.k, c.k, c.s, c.s, c.p, c.p);
    std::vector<int8_t> packed(pb);
    pack_conv_weights_for(c.Cstore, c.OC, c.H, c.H, c.k, c.k, c.s, c.s, c.p, c.p, q.data(), c.IC, packed.data());
    std::vector<float> alpha(ocp, 0.f), beta(ocp, 0.f);
    fold_bn(m->scales.at(c.in_site), sw.data(), m->tensors.at(c.bn + ".weight").data(),
            m->tensors.at(c.bn + ".bias").data(), m->tensors.at(c.bn + ".running_mean").data(),
            m->tensors.at(c.bn + ".running_var").data(), 1e-5f, m->scales.at(c.site), c.OC, alpha.data(),
            beta.data());
    if ((rc = dev_alloc(m, &c.w, pb)) || (rc = dev_alloc(m, &c.alpha, ocp * 4)) ||
        (rc = dev_alloc(m, &c.beta, ocp * 4)))
      return rc;
    hipError_t e;
    if ((e = hipMemcpy(c.w, packed.data(), pb, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(c.alpha, alpha.data(), ocp * 4, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(c.beta, beta.data(), ocp * 4, hipMemcpyHostToDevice)) != hipSuccess)
      return hip_fail(e, "weight upload");
    if (c.k == 1 && c.s == 2 && c.Cstore % 32 == 0) {  // downsample: fused into the stride-2 conv1
      std::vector<int8_t> fp(downsample_packed_bytes(c.OC, c.Cstore));
      downsample_pack(q.data(), c.OC, c.IC, c.Cstore, fp.data());
      if ((rc = dev_alloc(m, &c.wf, fp.size()))) return rc;
      if ((e = hipMemcpy(c.wf, fp.data(), fp.size(), hipMemcpyHostToDevice)) != hipSuccess)
        return hip_fail(e, "downsample weight upload");
    }
    if (&c == &m->convs[m->stem]) {  // the fused stem's space-to-depth weight image
      std::vector<int8_t> sp(stem_packed_bytes());
      std::vector<float> sa(64);
      pack_stem_weights(q.data(), alpha.data(), sp.data(), sa.data());
      if ((rc = dev_alloc(m, &m->stem_w, sp.size())) || (rc = dev_alloc(m, &m->stem_alpha, 64 * 4))) return rc;
      if ((e = hipMemcpy(m->stem_w, sp.data(), sp.size(), hipMemcpyHostToDevice)) != hipSuccess ||
          (e = hipMemcpy(m->stem_alpha, sa.data(), 64 * 4, hipMemcpyHostToDevice)) != hipSuccess)
        return hip_fail(e, "stem weight upload");
    }
  }
  {  // FC: int8 [1000][512] per-row scales; logits = fmaf(acc, s_gap*s_w[o], bias[o])
    const int O = 1000, I = 512, op = packed_oc(O);
    std::vector<int8_t> q;
    std::vector<float> sw;
    weights_s8(m, "fc.weight", O, I, q, sw);
    std::vector<int8_t> packed(packed_bytes(O, I, 1, 1));
    pack_conv_weights(q.data(), O, I, 1, 1, I, packed.data());
    std::vector<float> alpha(op, 0.f), beta(op, 0.f);
    const float sg = m->scales.at("gap");
    const std::vector<float>& bias = m->tensors.at("fc.bias");
    for (int o = 0; o < O; ++o) {
      alpha[o] = sg * sw[o];
      beta[o] = bias[o];
    }
    if ((rc = dev_alloc(m, &m->fc_w, packed.size())) || (rc = dev_alloc(m, &m->fc_alpha, op * 4)) ||
        (rc = dev_alloc(m, &m->fc_beta, op * 4)))
      return rc;
    hipError_t e;
    if ((e = hipMemcpy(m->fc_w, packed.data(), packed.size(), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(m->fc_alpha, alpha.data(), op * 4, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(m->fc_beta, beta.data(), op * 4, hipMemcpyHostToDevice)) != hipSuccess)
      return hip_fail(e, "fc upload");
  }
  // Workspace (int8 NHWC), sized once for max_batch.
  const size_t B = (size_t)max_batch;
  if ((rc = dev_alloc(m, &m->gq, B * 512))) return rc;
  for (auto& b : m->buf)
    if ((rc = dev_alloc(m, &b, B * 56 * 56 * 64))) return rc;
  if (m->keep) {
    const std::pair<const char*, size_t> kb[] = {{"stem_pool", 56 * 56 * 64}, {"layer1", 56 * 56 * 64},
                                                 {"layer2", 28 * 28 * 128}, {"layer3", 14 * 14 * 256},
                                                 {"layer4", 7 * 7 * 512}};
    for (const auto& k : kb) {
      int8_t* p = nullptr;
      if ((rc = dev_alloc(m, &p, B * k.second))) return rc;
      m->keepbuf[k.first] = p;
    }
  }
  (void)s;
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return hip_fail(e, "prepare sync");
  m->max_batch = max_batch;
  m->prepared = true;
  return DLQ_OK;
}

int dlq_basic_block_s8(dlq_resnet18* m, int block, const int8_t* x, int N, int8_t* y, void* stream) {
  if (!m) return fail(DLQ_ERR_ARG, "basic_block: null model");
  if (!m->prepared) return fail(DLQ_ERR_STATE, "basic_block: call dlq_resnet18_prepare first");
  if (block < 0 || block >= (int)m->blocks.size()) return fail(DLQ_ERR_ARG, "basic_block: block index out of range");
  if (N < 0 || N > m->max_batch) return fail(DLQ_ERR_ARG, "basic_block: batch exceeds prepared max_batch");
  if (N == 0) return DLQ_OK;
  if (!x || !y) return fail(DLQ_ERR_ARG, "basic_block: null pointer");
  if (m->prec != DLQ_PREC_INT8) return fail(DLQ_ERR_STATE, "basic_block: int8 models only");
  const Block& b = m->blocks[block];
  const int H = m->convs[b.c1].H;
  int OH, OW;
  // intermediates in two of the engine's activation buffers (not re-entrant with forward)
  return basic_block_forward(m, b, x, N, H, H, m->buf[2], m->buf[3], y, (hipStream_t)stream, &OH, &OW);
}

namespace {

// One forward pass over images [img0, img0 + B) of the workspace partition
// starting at image img0 (every buffer is sized max_batch x the largest
// per-image activation, so partitions of disjoint image ranges never overlap).
// fp8 conv launch (generic implicit-GEMM kernel, e4m3 in and out).
int conv_f8(dlq_resnet18* m, const ConvLayer& c, const int8_t* x, int N, int H, const int8_t* residual,
            float s_res, bool relu, int8_t* y, hipStream_t s) {
  const bool wide = f8_wide(c.Cstore, c.OC, H, H, c.k, c.k, c.s, c.s, c.p, c.p);
  int rc = mark(m, s, wide ? DLQ_FAM_WIDE : DLQ_FAM_F8);
  if (rc) return rc;
  dlq_conv_desc d{N, H, H, c.Cstore, c.OC, c.k, c.k, c.s, c.s, c.p, c.p};
  const float r_s = residual ? dlq::res_scale(s_res, m->scales.at(c.site)) : 0.f;
  return dlq_conv2d_nhwc_f8(&d, (const uint8_t*)x, (const uint8_t*)c.w, c.alpha, c.beta, (const uint8_t*)residual,
                            r_s, relu ? 1 : 0, (uint8_t*)y, s);
}

// The fp8 forward (oracle.py resnet18_forward_f8): quantise -> conv1 ->
// maxpool -> 8 blocks of 2-3 conv launches -> GAP -> FC.
int forward_pass_f8(dlq_resnet18* m, const float* x, int B, float* logits, hipStream_t s, bool record) {
  const size_t nB = (size_t)B;
  int rc;
  const ConvLayer& st = m->convs[m->stem];
  int ci = 0;
  int8_t* cur = m->buf[ci];
  if ((rc = mark(m, s, DLQ_FAM_STEM))) return rc;
  rc = dlq_stem_fused_f8(x, B, (const uint8_t*)m->stem_w, m->stem_alpha, st.beta, inv_scale(m->scales.at("input")),
                         (uint8_t*)cur, s);
  if (rc) return rc;
  if (record && (rc = record_stage(m, "stem_pool", cur, nB * 56 * 56 * 64, s))) return rc;
  int H = 56;
  for (const Block& b : m->blocks) {
    int fi[3], k = 0;
    for (int i = 0; i < 4; ++i)
      if (i != ci && k < 3) fi[k++] = i;
    const ConvLayer& c1 = m->convs[b.c1];
    const ConvLayer& c2 = m->convs[b.c2];
    int8_t *h = m->buf[fi[0]], *dsb = m->buf[fi[1]], *out = m->buf[fi[2]];
    if (fused_l1_block(m, b, H, H)) {  // both convs, the identity add and the ReLUs in one launch
      if ((rc = mark(m, s, DLQ_FAM_L1))) return rc;
      const float r_s = dlq::res_scale(m->scales.at(c1.in_site), m->scales.at(c2.site));
      rc = dlq_block_l1_nhwc_f8((const uint8_t*)cur, B, (const uint8_t*)c1.w, c1.alpha, c1.beta, (const uint8_t*)c2.w,
                                c2.alpha, c2.beta, r_s, (uint8_t*)out, s);
      if (rc) return rc;
      ci = fi[2];
      cur = out;
      if (record && b.name.size() == 8 && b.name[7] == '1')
        if ((rc = record_stage(m, b.name.substr(0, 6).c_str(), cur, nB * H * H * b.oc, s))) return rc;
      continue;
    }
    const int8_t* skip = cur;
    float s_skip = m->scales.at(c1.in_site);
    if (b.down && m->convs[b.ds].wf && f8_wide(c1.Cstore, c1.OC, H, H, 3, 3, 2, 2, 1, 1)) {
      // conv1 (3x3/s2) and the 1x1/s2 downsample in one launch
      const ConvLayer& ds = m->convs[b.ds];
      if ((rc = mark(m, s, DLQ_FAM_S2DS))) return rc;
      dlq_conv_desc d{B, H, H, c1.Cstore, c1.OC, 3, 3, 2, 2, 1, 1};
      rc = dlq_conv2d_s2_ds_nhwc_f8(&d, (const uint8_t*)cur, (const uint8_t*)c1.w, c1.alpha, c1.beta,
                                    (const uint8_t*)ds.wf, ds.alpha, ds.beta, (uint8_t*)h, (uint8_t*)dsb, s);
      if (rc) return rc;
      skip = dsb;
      s_skip = m->scales.at(ds.site);
    } else if ((rc = conv_f8(m, c1, cur, B, H, nullptr, 0.f, true, h, s))) {
      return rc;
    } else if (b.down) {
      const ConvLayer& ds = m->convs[b.ds];
      if ((rc = conv_f8(m, ds, cur, B, H, nullptr, 0.f, false, dsb, s))) return rc;
      skip = dsb;
      s_skip = m->scales.at(ds.site);
    }
    const int OH = out_dim(H, 3, c1.s, 1);
    if ((rc = conv_f8(m, c2, h, B, OH, skip, s_skip, true, out, s))) return rc;
    ci = fi[2];
    cur = out;
    H = OH;
    if (record && b.name.size() == 8 && b.name[7] == '1')
      if ((rc = record_stage(m, b.name.substr(0, 6).c_str(), cur, nB * H * H * b.oc, s))) return rc;
  }
  const std::string last = m->convs[m->blocks.back().c2].site;
  // gap_k * 2^-9 (oracle.py gap_k_f8): the sums are in e4m3 units of 2^-9
  const float k = ((m->scales.at(last) / (float)(H * H)) / m->scales.at("gap")) * 0x1p-9f;
  if ((rc = mark(m, s, DLQ_FAM_GAP))) return rc;
  if ((rc = dlq_gap_nhwc_f8((const uint8_t*)cur, B, 512, H * H, k, (uint8_t*)m->gq, s))) return rc;
  if (record) m->stage["gap"] = {m->gq, nB * 512};
  if ((rc = mark(m, s, DLQ_FAM_FC))) return rc;
  rc = dlq_linear_f8((const uint8_t*)m->gq, B, 512, (const uint8_t*)m->fc_w, 1000, m->fc_alpha, m->fc_beta, logits, s);
  if (rc) return rc;
  return mark(m, s, -1);
}

int forward_pass(dlq_resnet18* m, const float* x, int B, float* logits, hipStream_t s, size_t img0,
                 bool record) {
  if (m->prec == DLQ_PREC_FP8) return forward_pass_f8(m, x, B, logits, s, record);
  const size_t nB = (size_t)B;
  constexpr size_t kAct = 56 * 56 * 64;  // largest per-image activation (buffer stride per image)
  void* stream = s;
  int rc;
  int H = 56, W = 56;
  int ci = 0;  // index of the buffer holding the current activation
  auto bufp = [&](int i) { return m->buf[i] + img0 * kAct; };
  int8_t* cur = bufp(ci);
  int8_t* gq = m->gq + img0 * 512;
  const ConvLayer& st = m->convs[m->stem];
  // 0+1) fused stem: quantise + conv 7x7/s2 + BN + ReLU + maxpool 3x3/s2
  //      (infer_e2e.cu:255-293) in one launch
  if ((rc = mark(m, s, DLQ_FAM_STEM))) return rc;
  if (B > 0) {  // (the stem's C-ABI entry, dlq_stem_fused_s8, with the next launch's prefetch)
    const Prefetch pf = block_prefetch(m, m->blocks[0], 56);
    hipError_t e = launch_stem_fused(x, B, m->stem_w, m->stem_alpha, st.beta, inv_scale(m->scales.at("input")), cur,
                                     s, false, prefetch_on() ? &pf : nullptr);
    if (e != hipSuccess) return hip_fail(e, "stem launch");
  }
  if (record && (rc = record_stage(m, "stem_pool", cur, nB * H * W * 64, s))) return rc;
  // 2-5) layer1..layer4 (:300-415)
  bool pooled = false;  // the last conv wrote the GAP codes (gap_epi)
  for (size_t bi = 0; bi < m->blocks.size(); ++bi) {
    const Block& b = m->blocks[bi];
    int fi[3];
    int k = 0;
    for (int i = 0; i < 4; ++i)
      if (i != ci && k < 3) fi[k++] = i;
    int OH, OW;
    // the launch after this block: the next block's first launch, or the
    // head's FC weights
    Prefetch next{};
    if (bi + 1 < m->blocks.size()) {
      next = block_prefetch(m, m->blocks[bi + 1], b.stride == 2 ? out_dim(H, 3, 2, 1) : H);
    } else {
      next.p[0] = m->fc_w;
      next.n[0] = 1;
      next.stride[0] = 0;
      next.len[0] = (int)(packed_bytes(1000, 512, 1, 1) & ~(size_t)1023);
    }
    // the last block's conv2 pools its own output (its H is the block's input
    // H: layer4.1 keeps the resolution) when it is the wide 7x7x512 conv
    int8_t* gap_y = nullptr;
    float gap_k = 0.f;
    if (bi + 1 == m->blocks.size() && gap_epi_on() && !head_split() && b.stride == 1 && !b.down) {
      const ConvLayer& c2 = m->convs[b.c2];
      if (H == 7 && W == 7 && c2.Cstore == 512 && c2.OC == 512 && conv3x3w_shape(512, 512, 7, 7, 3, 3, 1, 1, 1, 1)) {
        gap_y = gq;
        gap_k = (m->scales.at(c2.site) / (float)(H * W)) / m->scales.at("gap");
      }
    }
    rc = basic_block_forward(m, b, cur, B, H, W, bufp(fi[0]), bufp(fi[1]), bufp(fi[2]), s, &OH, &OW, &next, gap_y,
                             gap_k);
    if (rc) return rc;
    pooled = gap_y != nullptr;
    ci = fi[2];
    cur = bufp(ci);
    H = OH;
    W = OW;
    if (record && b.name.size() == 8 && b.name[7] == '1')
      if ((rc = record_stage(m, b.name.substr(0, 6).c_str(), cur, nB * H * W * b.oc, s))) return rc;
  }
  // 6) GAP + FC (:417-433)
  const std::string last = m->convs[m->blocks.back().c2].site;
  const float k = (m->scales.at(last) / (float)(H * W)) / m->scales.at("gap");
  if (pooled) {  // the last conv wrote the GAP codes: the FC alone
    if (record) m->stage["gap"] = {gq, nB * 512};
    if ((rc = mark(m, s, DLQ_FAM_FC))) return rc;
    rc = dlq_linear_s8(gq, B, 512, m->fc_w, 1000, m->fc_alpha, m->fc_beta, 0, DLQ_OUT_F32, logits, stream);
    if (rc) return rc;
    return mark(m, s, -1);
  }
  if ((rc = mark(m, s, DLQ_FAM_GAP))) return rc;
  if (!m->keep && !head_split()) {  // one launch (head.hip gap_fc_kernel); the GAP codes stay on chip
    rc = dlq_gap_fc_s8(cur, B, 512, H * W, k, m->fc_w, 1000, m->fc_alpha, m->fc_beta, logits, stream);
    if (rc) return rc;
    return mark(m, s, -1);
  }
  rc = dlq_gap_nhwc_s8(cur, B, 512, H * W, k, gq, stream);
  if (rc) return rc;
  if (record) m->stage["gap"] = {gq, nB * 512};
  if ((rc = mark(m, s, DLQ_FAM_FC))) return rc;
  rc = dlq_linear_s8(gq, B, 512, m->fc_w, 1000, m->fc_alpha, m->fc_beta, 0, DLQ_OUT_F32, logits, stream);
  if (rc) return rc;
  return mark(m, s, -1);
}

// Split a batch into two halves on two streams (DLQ_SPLIT=1; measured within
// 1% of the single stream at B=256, so off by default)?  Never while timing
// launches (the per-launch events assume one stream) or keeping stage dumps,
// and only for batches big enough that a half still fills the chip.
bool use_split(const dlq_resnet18* m, int B) {
  static const bool on = [] {
    const char* e = std::getenv("DLQ_SPLIT");
    return e && e[0] == '1';
  }();
  return on && m->prec == DLQ_PREC_INT8 && !m->timing && !m->keep && B >= 64;
}

// Replay the forward as a hipGraph?  Only with knob "graph" = 1 (DLQ_GRAPH=1
// or dlq_set_knob): measured at B=256 the replay is ~1 % SLOWER than the 16
// direct launches (409k vs 414k images/s, same box), so direct launches are
// the default.  Never while timing launches (events between launches) or
// keeping stage dumps (host-side copies).
bool use_graph(const dlq_resnet18* m) {
  return g_knob_graph.load(std::memory_order_relaxed) == 1 && !m->timing && !m->keep;
}

int forward_graph(dlq_resnet18* m, const float* x, int B, float* logits, hipStream_t s) {
  hipError_t e = hipSuccess;
  const unsigned gen = g_knob_gen.load(std::memory_order_relaxed);
  if (!m->gexec || m->g_x != x || m->g_B != B || m->g_logits != logits || m->g_gen != gen) {
    drop_graph(m);
    if (!m->gs && (e = hipStreamCreateWithFlags(&m->gs, hipStreamNonBlocking)) != hipSuccess)
      return hip_fail(e, "graph stream");
    if ((e = hipStreamBeginCapture(m->gs, hipStreamCaptureModeRelaxed)) != hipSuccess)
      return hip_fail(e, "hipStreamBeginCapture");
    int rc = forward_pass(m, x, B, logits, m->gs, 0, true);
    hipGraph_t g = nullptr;
    e = hipStreamEndCapture(m->gs, &g);
    if (rc) {
      if (g) (void)hipGraphDestroy(g);
      return rc;
    }
    if (e != hipSuccess) return hip_fail(e, "hipStreamEndCapture");
    e = hipGraphInstantiate(&m->gexec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) {
      m->gexec = nullptr;
      return hip_fail(e, "hipGraphInstantiate");
    }
    m->g_x = x;
    m->g_gen = gen;
    m->g_B = B;
    m->g_logits = logits;
  }
  if ((e = hipGraphLaunch(m->gexec, s)) != hipSuccess) return hip_fail(e, "hipGraphLaunch");
  return DLQ_OK;
}

}  // namespace

int dlq_resnet18_forward(dlq_resnet18* m, const float* x, int B, float* logits, void* stream) {
  if (!m) return fail(DLQ_ERR_ARG, "forward: null model");
  if (!m->prepared) return fail(DLQ_ERR_STATE, "forward: call dlq_resnet18_prepare first");
  if (B < 0 || B > m->max_batch) return fail(DLQ_ERR_ARG, "forward: batch exceeds prepared max_batch");
  if (B == 0) return DLQ_OK;  // empty batch: nothing to read or write
  if (!x || !logits) return fail(DLQ_ERR_ARG, "forward: null argument");
  hipStream_t s = (hipStream_t)stream;
  int rc;
  if (use_graph(m) && !use_split(m, B)) {
    const bool fresh = !m->gexec || m->g_x != x || m->g_B != B || m->g_logits != logits;
    if (fresh) m->stage.clear();  // capture re-records the stage pointers; a replay writes the same buffers
    if ((rc = forward_graph(m, x, B, logits, s))) return rc;
    m->last_B = B;
    return DLQ_OK;
  }
  m->stage.clear();
  if (!use_split(m, B)) {
    if ((rc = forward_pass(m, x, B, logits, s, 0, true))) return rc;
  } else {
    hipError_t e = hipSuccess;
    if (!m->s2) {
      if ((e = hipStreamCreateWithFlags(&m->s2, hipStreamNonBlocking)) != hipSuccess ||
          (e = hipEventCreateWithFlags(&m->fork, hipEventDisableTiming)) != hipSuccess ||
          (e = hipEventCreateWithFlags(&m->join, hipEventDisableTiming)) != hipSuccess)
        return hip_fail(e, "split stream setup");
    }
    const int h1 = B / 2, h2 = B - h1;
    if ((e = hipEventRecord(m->fork, s)) != hipSuccess || (e = hipStreamWaitEvent(m->s2, m->fork, 0)) != hipSuccess)
      return hip_fail(e, "split fork");
    if ((rc = forward_pass(m, x + (size_t)h1 * 3 * 224 * 224, h2, logits + (size_t)h1 * 1000, m->s2, h1, false)))
      return rc;
    if ((rc = forward_pass(m, x, h1, logits, s, 0, false))) return rc;
    if ((e = hipEventRecord(m->join, m->s2)) != hipSuccess || (e = hipStreamWaitEvent(s, m->join, 0)) != hipSuccess)
      return hip_fail(e, "split join");
  }
  m->last_B = B;
  return DLQ_OK;
}

int dlq_resnet18_set_timing(dlq_resnet18* m, int on) {
  if (!m) return fail(DLQ_ERR_ARG, "set_timing: null");
  m->timing = on != 0;
  m->ev_used = 0;
  drop_graph(m);
  return DLQ_OK;
}

int dlq_resnet18_timing(dlq_resnet18* m, double* ms, int* launches, int* forwards) {
  if (!m || !ms || !launches) return fail(DLQ_ERR_ARG, "timing: null");
  for (int f = 0; f < DLQ_FAM_COUNT; ++f) {
    ms[f] = 0.0;
    launches[f] = 0;
  }
  int nf = 0;
  if (m->ev_used > 0) {
    hipError_t he = hipEventSynchronize(m->ev[m->ev_used - 1]);
    if (he != hipSuccess) return hip_fail(he, "hipEventSynchronize");
  }
  for (size_t i = 0; i + 1 < m->ev_used; ++i) {
    const int f = m->ev_tag[i];
    if (f < 0) continue;  // end of one forward -> start of the next
    float t = 0;
    hipError_t he = hipEventElapsedTime(&t, m->ev[i], m->ev[i + 1]);
    if (he != hipSuccess) return hip_fail(he, "hipEventElapsedTime");
    ms[f] += t;
    launches[f] += 1;
  }
  for (size_t i = 0; i < m->ev_used; ++i) nf += m->ev_tag[i] < 0;
  if (forwards) *forwards = nf;
  m->ev_used = 0;
  return DLQ_OK;
}

int dlq_resnet18_family_work(const dlq_resnet18* m, double* macs, double* bytes) {
  if (!m || !macs || !bytes) return fail(DLQ_ERR_ARG, "family_work: null");
  for (int f = 0; f < DLQ_FAM_COUNT; ++f) macs[f] = bytes[f] = 0.0;
  if (m->prec == DLQ_PREC_FP8) {  // stem, layer1 blocks, s2 + downsample, conv3x3i<F8> (wide), GAP, FC
    auto fam = [&](const ConvLayer& c) {
      return f8_wide(c.Cstore, c.OC, c.H, c.H, c.k, c.k, c.s, c.s, c.p, c.p) ? DLQ_FAM_WIDE : DLQ_FAM_F8;
    };
    for (const Block& b : m->blocks) {  // fused layer1 blocks: block input + output bytes
      if (!fused_l1_block(m, b, m->convs[b.c1].H, m->convs[b.c1].H)) continue;
      const ConvLayer& c1 = m->convs[b.c1];
      macs[DLQ_FAM_L1] += 2.0 * c1.OC * c1.IC * 9 * c1.H * c1.H;
      bytes[DLQ_FAM_L1] += 2.0 * c1.H * c1.H * c1.OC;
    }
    auto in_l1 = [&](const ConvLayer& c) {
      for (const Block& b : m->blocks)
        if ((&c == &m->convs[b.c1] || &c == &m->convs[b.c2]) && fused_l1_block(m, b, m->convs[b.c1].H, m->convs[b.c1].H))
          return true;
      return false;
    };
    // 0: not in a fused stride-2 launch, 1: its 3x3 conv1, 2: its downsample
    auto in_s2ds = [&](const ConvLayer& c) {
      for (const Block& b : m->blocks) {
        if (!b.down || !m->convs[b.ds].wf) continue;
        const ConvLayer& c1 = m->convs[b.c1];
        if (!f8_wide(c1.Cstore, c1.OC, c1.H, c1.H, 3, 3, 2, 2, 1, 1)) continue;
        if (&c == &c1) return 1;
        if (&c == &m->convs[b.ds]) return 2;
      }
      return 0;
    };
    for (const ConvLayer& c : m->convs) {
      const int OH = out_dim(c.H, c.k, c.s, c.p);
      if (in_l1(c)) continue;
      if (const int k = in_s2ds(c)) {  // one launch: the shared input once, both outputs
        macs[DLQ_FAM_S2DS] += (double)c.OC * c.IC * c.k * c.k * OH * OH;
        bytes[DLQ_FAM_S2DS] += (k == 1 ? (double)c.H * c.H * c.Cstore : 0.0) + (double)OH * OH * c.OC;
        continue;
      }
      if (&c == &m->convs[m->stem]) {  // fp32 input read + pooled e4m3 output
        macs[DLQ_FAM_STEM] = (double)c.OC * c.IC * c.k * c.k * OH * OH;
        bytes[DLQ_FAM_STEM] = 3.0 * 224 * 224 * 4 + 56.0 * 56 * 64;
        continue;
      }
      macs[fam(c)] += (double)c.OC * c.IC * c.k * c.k * OH * OH;
      bytes[fam(c)] += (double)c.H * c.H * c.Cstore + (double)OH * OH * c.OC;
    }
    for (const Block& b : m->blocks) {  // conv2's residual read
      const ConvLayer& c2 = m->convs[b.c2];
      if (!in_l1(c2)) bytes[fam(c2)] += (double)c2.H * c2.H * c2.OC;
    }
    macs[DLQ_FAM_FC] = 512.0 * 1000;
    bytes[DLQ_FAM_FC] = 512.0 + 4000.0;
    bytes[DLQ_FAM_GAP] = 7.0 * 7 * 512 + 512;
    return DLQ_OK;
  }
  // stem: fp32 input read + pooled int8 output written, 7x7x3 MACs at 112x112
  const ConvLayer& st = m->convs[m->stem];
  macs[DLQ_FAM_STEM] = (double)st.OC * st.IC * st.k * st.k * 112.0 * 112.0;
  bytes[DLQ_FAM_STEM] = 3.0 * 224 * 224 * 4 + 56.0 * 56 * 64;
  for (const Block& b : m->blocks) {
    const ConvLayer& c1 = m->convs[b.c1];
    const ConvLayer& c2 = m->convs[b.c2];
    const int H = c1.H, OH = c2.H;
    const double mac1 = (double)c1.OC * c1.IC * 9 * OH * OH, mac2 = (double)c2.OC * c2.IC * 9 * OH * OH;
    const double in1 = (double)H * H * c1.IC, out = (double)OH * OH * c2.OC;
    if (fused_l1_block(m, b, H, H)) {  // one launch: block input + output bytes
      macs[DLQ_FAM_L1] += mac1 + mac2;
      bytes[DLQ_FAM_L1] += in1 + out;
      continue;
    }
    if (b.down) {
      const ConvLayer& ds = m->convs[b.ds];
      macs[DLQ_FAM_S2DS] += mac1 + (double)ds.OC * ds.IC * OH * OH;
      bytes[DLQ_FAM_S2DS] += in1 + 2 * out;
    } else {
      macs[conv_family(c1, H)] += mac1;
      bytes[conv_family(c1, H)] += in1 + out;
    }
    macs[conv_family(c2, OH)] += mac2;
    bytes[conv_family(c2, OH)] += out + out + out;  // input, residual, output
  }
  if (head_split()) {
    macs[DLQ_FAM_FC] = 512.0 * 1000;
    bytes[DLQ_FAM_FC] = 512.0 + 4000.0;
    bytes[DLQ_FAM_GAP] = 7.0 * 7 * 512 + 512;
  } else {  // gap_fc_kernel: layer4 output in, fp32 logits out
    macs[DLQ_FAM_GAP] = 512.0 * 1000;
    bytes[DLQ_FAM_GAP] = 7.0 * 7 * 512 + 4000.0;
  }
  return DLQ_OK;
}

int dlq_resnet18_set_keep_stages(dlq_resnet18* m, int on) {
  if (!m) return fail(DLQ_ERR_ARG, "keep_stages: null");
  if ((on != 0) != m->keep) m->prepared = false;
  m->keep = on != 0;
  return DLQ_OK;
}

int dlq_resnet18_stage(dlq_resnet18* m, const char* name, void* dst, size_t cap, size_t* bytes,
                       void* stream) {
  if (!m || !name) return fail(DLQ_ERR_ARG, "stage: null argument");
  auto it = m->stage.find(name);
  if (it == m->stage.end()) return fail(DLQ_ERR_STATE, std::string("stage: not available: ") + name);
  if (bytes) *bytes = it->second.second;
  if (!dst) return DLQ_OK;
  if (cap < it->second.second) return fail(DLQ_ERR_ARG, "stage: destination too small");
  hipError_t e = hipMemcpyAsync(dst, it->second.first, it->second.second, hipMemcpyDeviceToDevice,
                                (hipStream_t)stream);
  return e == hipSuccess ? DLQ_OK : hip_fail(e, "stage copy");
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Reference-semantics fp32 forward (ref_f32.hip): infer_e2e.cu:259-438 op for
// op on the GPU, for activation-scale calibration and the launcher's --fp32
// mode.  Model preparation / parity, not the timed path: fp32 weights are
// uploaded per call (as the reference does, :262, :304-334) and freed after.
namespace {

struct DevArena {  // per-call device allocations, freed on scope exit
  std::vector<void*> p;
  ~DevArena() {
    for (void* q : p) (void)hipFree(q);
  }
  template <typename T>
  int alloc(T** out, size_t bytes) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, bytes ? bytes : 16);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc (fp32 forward)");
    p.push_back(q);
    *out = (T*)q;
    return DLQ_OK;
  }
  template <typename T>
  int upload(T** out, const T* src, size_t n, hipStream_t s) {
    int rc = alloc(out, n * sizeof(T));
    if (rc) return rc;
    // synchronous (on the stream): the host vectors behind src are
    // temporaries of the caller, and a pageable async copy is not guaranteed
    // to have staged them when the call returns
    hipError_t e = hipMemcpyAsync(*out, src, n * sizeof(T), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    return e == hipSuccess ? DLQ_OK : hip_fail(e, "fp32 weight upload");
  }
};

int check_tensors(const dlq_resnet18* m) {
  for (const auto& n : required_tensors(m))
    if (!m->tensors.count(n) && !m->qtensors.count(n)) return fail(DLQ_ERR_STATE, "missing tensor: " + n);
  return DLQ_OK;
}

// Sites in calibration order (dlq_amd/quant.py calibrate_resnet18).
std::vector<std::string> calib_sites(const dlq_resnet18* m) {
  std::vector<std::string> s = {"input", "conv1"};
  for (const Block& b : m->blocks) {
    s.push_back(b.name + ".conv1");
    if (b.down) s.push_back(b.name + ".downsample");
    s.push_back(b.name + ".conv2");
  }
  s.push_back("gap");
  return s;
}

int keep_f32(dlq_resnet18* m, const char* name, const float* src, size_t n, hipStream_t s) {
  auto it = m->stage_f32.find(name);
  if (it != m->stage_f32.end() && it->second.second != n * 4) {
    (void)hipFree(it->second.first);
    m->stage_f32.erase(it);
    it = m->stage_f32.end();
  }
  if (it == m->stage_f32.end()) {
    float* q = nullptr;
    hipError_t e = hipMalloc(&q, n * 4);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc (fp32 stage)");
    it = m->stage_f32.emplace(name, std::make_pair(q, n * 4)).first;
  }
  hipError_t e = hipMemcpyAsync(it->second.first, src, n * 4, hipMemcpyDeviceToDevice, s);
  return e == hipSuccess ? DLQ_OK : hip_fail(e, "fp32 stage copy");
}

// amax (host, per calib_sites order) may be null; logits may be null.
int ref_forward_f32(dlq_resnet18* m, const float* x, int B, float* logits, std::vector<float>* amax_out,
                    hipStream_t s) {
  int rc;
  if ((rc = check_tensors(m))) return rc;
  const std::vector<std::string> sites = calib_sites(m);
  auto site_ix = [&](const std::string& n) {
    for (size_t i = 0; i < sites.size(); ++i)
      if (sites[i] == n) return (int)i;
    return -1;
  };
  DevArena ar;
  unsigned* amax = nullptr;
  if ((rc = ar.alloc(&amax, sites.size() * 4))) return rc;
  hipError_t e = hipMemsetAsync(amax, 0, sites.size() * 4, s);
  if (e != hipSuccess) return hip_fail(e, "amax reset");
  // conv + BN parameters of one ConvLayer, uploaded
  struct DevConv {
    float *w, *g, *b, *mu, *d;
  };
  auto upload_conv = [&](const ConvLayer& c, DevConv& dc) {
    const int K = c.IC * c.k * c.k;
    const std::vector<float> w = weights_f32(m, c.wname, c.OC, K);
    std::vector<float> d(c.OC);
    const std::vector<float>& var = m->tensors.at(c.bn + ".running_var");
    for (int o = 0; o < c.OC; ++o) d[o] = std::sqrt(var[o] + 1e-5f);  // bn_inference.cu:22 (sqrtf(v + eps))
    int r;
    if ((r = ar.upload(&dc.w, w.data(), w.size(), s)) ||
        (r = ar.upload(&dc.g, m->tensors.at(c.bn + ".weight").data(), (size_t)c.OC, s)) ||
        (r = ar.upload(&dc.b, m->tensors.at(c.bn + ".bias").data(), (size_t)c.OC, s)) ||
        (r = ar.upload(&dc.mu, m->tensors.at(c.bn + ".running_mean").data(), (size_t)c.OC, s)) ||
        (r = ar.upload(&dc.d, d.data(), d.size(), s)))
      return r;
    return (int)DLQ_OK;
  };
  auto conv = [&](const ConvLayer& c, const float* in, int H, float* out, bool relu, const std::string& site) {
    DevConv dc;
    int r = upload_conv(c, dc);
    if (r) return r;
    const int ix = site.empty() ? -1 : site_ix(site);
    hipError_t he = launch_ref_conv_bn(in, B, c.IC, H, H, dc.w, c.OC, c.k, c.s, c.p, dc.g, dc.b, dc.mu, dc.d,
                                       relu ? 1 : 0, out, ix < 0 ? nullptr : amax + ix, s);
    return he == hipSuccess ? (int)DLQ_OK : hip_fail(he, "fp32 conv launch");
  };
  const size_t nB = (size_t)B;
  if ((e = launch_amax(x, (long)(nB * 3 * 224 * 224), amax + site_ix("input"), s)) != hipSuccess)
    return hip_fail(e, "amax launch");
  float *c1, *buf[4];
  if ((rc = ar.alloc(&c1, nB * 64 * 112 * 112 * 4))) return rc;
  for (auto& b : buf)
    if ((rc = ar.alloc(&b, nB * 64 * 56 * 56 * 4))) return rc;
  // stem: conv1 -> bn1 -> relu -> maxpool (:255-293)
  if ((rc = conv(m->convs[m->stem], x, 224, c1, true, "conv1"))) return rc;
  if ((e = launch_ref_maxpool(c1, B * 64, 112, 112, buf[0], s)) != hipSuccess) return hip_fail(e, "maxpool launch");
  if ((rc = keep_f32(m, "stem_pool", buf[0], nB * 64 * 56 * 56, s))) return rc;
  int ci = 0, H = 56;
  for (const Block& b : m->blocks) {  // basic_block_forward (:156-203)
    int fi[3], k = 0;
    for (int i = 0; i < 4; ++i)
      if (i != ci && k < 3) fi[k++] = i;
    float *in = buf[ci], *h = buf[fi[0]], *dsb = buf[fi[1]], *out = buf[fi[2]];
    const ConvLayer& c1l = m->convs[b.c1];
    const ConvLayer& c2l = m->convs[b.c2];
    const int OH = out_dim(H, 3, c1l.s, 1);
    if ((rc = conv(c1l, in, H, h, true, b.name + ".conv1"))) return rc;
    if ((rc = conv(c2l, h, OH, out, false, ""))) return rc;
    const float* skip = in;
    if (b.down) {
      if ((rc = conv(m->convs[b.ds], in, H, dsb, false, b.name + ".downsample"))) return rc;
      skip = dsb;
    }
    const long n = (long)nB * b.oc * OH * OH;
    if ((e = launch_ref_add_relu(out, skip, n, amax + site_ix(b.name + ".conv2"), s)) != hipSuccess)
      return hip_fail(e, "add_relu launch");
    ci = fi[2];
    H = OH;
    if (b.name.size() == 8 && b.name[7] == '1')
      if ((rc = keep_f32(m, b.name.substr(0, 6).c_str(), out, (size_t)n, s))) return rc;
  }
  float *gap, *fw, *fb, *lg;
  if ((rc = ar.alloc(&gap, nB * 512 * 4)) || (rc = ar.alloc(&lg, nB * 1000 * 4))) return rc;
  if ((e = launch_ref_gap(buf[ci], B * 512, H * H, gap, amax + site_ix("gap"), s)) != hipSuccess)
    return hip_fail(e, "gap launch");
  if ((rc = keep_f32(m, "gap", gap, nB * 512, s))) return rc;
  const std::vector<float> fcw = weights_f32(m, "fc.weight", 1000, 512);
  if ((rc = ar.upload(&fw, fcw.data(), fcw.size(), s)) ||
      (rc = ar.upload(&fb, m->tensors.at("fc.bias").data(), (size_t)1000, s)))
    return rc;
  if ((e = launch_ref_fc(gap, B, fw, fb, 1000, 512, lg, s)) != hipSuccess) return hip_fail(e, "fc launch");
  if ((rc = keep_f32(m, "logits", lg, nB * 1000, s))) return rc;
  if (logits && (e = hipMemcpyAsync(logits, lg, nB * 4000, hipMemcpyDeviceToDevice, s)) != hipSuccess)
    return hip_fail(e, "logits copy");
  std::vector<unsigned> am(sites.size());
  if ((e = hipMemcpyAsync(am.data(), amax, am.size() * 4, hipMemcpyDeviceToHost, s)) != hipSuccess ||
      (e = hipStreamSynchronize(s)) != hipSuccess)  // the arena is freed on return
    return hip_fail(e, "fp32 forward sync");
  if (amax_out) {
    amax_out->resize(am.size());
    for (size_t i = 0; i < am.size(); ++i) {
      float f;
      std::memcpy(&f, &am[i], 4);
      (*amax_out)[i] = f;
    }
  }
  return DLQ_OK;
}

}  // namespace

extern "C" {

int dlq_resnet18_forward_f32(dlq_resnet18* m, const float* x, int B, float* logits, void* stream) {
  if (!m || B < 0) return fail(DLQ_ERR_ARG, "forward_f32: bad args");
  if (B == 0) return DLQ_OK;
  if (!x) return fail(DLQ_ERR_ARG, "forward_f32: null input");
  return ref_forward_f32(m, x, B, logits, nullptr, (hipStream_t)stream);
}

int dlq_resnet18_calibrate(dlq_resnet18* m, const float* x, int B, float qmax, void* stream) {
  if (!m || B <= 0 || !x || !(qmax > 0.f)) return fail(DLQ_ERR_ARG, "calibrate: bad args");
  std::vector<float> amax;
  int rc = ref_forward_f32(m, x, B, nullptr, &amax, (hipStream_t)stream);
  if (rc) return rc;
  const std::vector<std::string> sites = calib_sites(m);
  for (size_t i = 0; i < sites.size(); ++i) {
    // dlq_amd/quant.py: float32(max(amax, 1e-8) / qmax), the quotient in double
    const double a = (double)amax[i] > 1e-8 ? (double)amax[i] : 1e-8;
    if ((rc = dlq_resnet18_set_scale(m, sites[i].c_str(), (float)(a / (double)qmax)))) return rc;
  }
  return DLQ_OK;
}

int dlq_resnet18_stage_f32(dlq_resnet18* m, const char* name, void* dst, size_t cap, size_t* bytes, void* stream) {
  if (!m || !name) return fail(DLQ_ERR_ARG, "stage_f32: null argument");
  auto it = m->stage_f32.find(name);
  if (it == m->stage_f32.end()) return fail(DLQ_ERR_STATE, std::string("stage_f32: not available: ") + name);
  if (bytes) *bytes = it->second.second;
  if (!dst) return DLQ_OK;
  if (cap < it->second.second) return fail(DLQ_ERR_ARG, "stage_f32: destination too small");
  hipError_t e = hipMemcpyAsync(dst, it->second.first, it->second.second, hipMemcpyDeviceToDevice, (hipStream_t)stream);
  return e == hipSuccess ? DLQ_OK : hip_fail(e, "stage_f32 copy");
}

int dlq_resnet18_macs_per_image(const dlq_resnet18* m, double* conv_macs, double* fc_macs) {
  if (!m) return fail(DLQ_ERR_ARG, "macs: null");
  double cm = 0;
  int H = 224;
  // stem
  {
    const auto& c = m->convs[m->stem];
    const int oh = out_dim(H, c.k, c.s, c.p);
    cm += (double)c.OC * c.IC * c.k * c.k * oh * oh;
    H = out_dim(oh, 3, 2, 1);
  }
  for (const auto& b : m->blocks) {
    const auto& c1 = m->convs[b.c1];
    const int oh = out_dim(H, c1.k, c1.s, c1.p);
    cm += (double)c1.OC * c1.IC * 9 * oh * oh;
    cm += (double)b.oc * b.oc * 9 * oh * oh;
    if (b.down) cm += (double)b.oc * b.ic * oh * oh;
    H = oh;
  }
  if (conv_macs) *conv_macs = cm;
  if (fc_macs) *fc_macs = 1000.0 * 512.0;
  return DLQ_OK;
}

}  // extern "C"
