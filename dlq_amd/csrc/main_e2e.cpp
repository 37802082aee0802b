// main_e2e.cpp -- bin/dlq_e2e, the C++ launcher of the int8 path.
//
// Reproduces the reference launcher's CLI and output contract
// (CUDA/resnet18-kernel-lab/cpp/fp32/runtime/infer_e2e.cu:221-441; the
// repository's main.cu is an empty file): reads the fp32 state_dict export
// (--manifest DIR, files <name>.bin as written by tools/export_resnet18.py),
// the fp32 NCHW input (--input X.bin, 1x3x224x224 as written by
// tools/preprocess_to_bin.py), runs ResNet-18 through the C ABI and prints
//   [E2E] top-1 class index = <i>, logit=<v>
// which tools/bench_fp32_vs_torch_e2e.py:51 parses.  --dump_dir writes the
// same checkpoint files as :297-433 (stem_pool, layer1..4, gap, logits) as
// fp32 NCHW (int8 stages dequantised with their scale) so
// tools/diag_e2e_compare.py can compare them.
// The reference's exact argv works: `--manifest DIR --input X.bin
// [--dump_dir D]` (what tools/bench_fp32_vs_torch_e2e.py:105 builds).  The
// int8 activation scales come from --scales FILE, else DIR/scales.txt (the
// manifest writers put it there), else they are calibrated once on the input
// by the reference-semantics fp32 forward on the GPU (dlq_resnet18_calibrate).
// Additions: --save_scales FILE, --fp32 (run the reference's fp32 forward op
// for op instead of the int8 engine; dumps in the same format), --batch B
// (replicate the image), --iters/--warmup (hipEvent timing).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/dlq.h"

#define CHECK_DLQ(x)                                                      \
  do {                                                                    \
    int rc_ = (x);                                                        \
    if (rc_ != DLQ_OK) {                                                  \
      std::fprintf(stderr, "dlq error %d at %s:%d: %s\n", rc_, __FILE__, \
                   __LINE__, dlq_last_error());                           \
      return 3;                                                           \
    }                                                                     \
  } while (0)
#define CHECK_HIP(x)                                                          \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, \
                   __LINE__);                                                 \
      return 3;                                                               \
    }                                                                         \
  } while (0)

static void usage() {
  std::printf(
      "dlq_e2e --manifest <dir> --input <input.bin> [--dump_dir <dir>]\n"
      "        [--scales <scales.txt>] [--save_scales <file>] [--fp32] [--batch B] [--iters K] [--warmup W]\n");
}

static bool load_f32(const std::string& path, std::vector<float>& v, size_t expect) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  f.seekg(0, std::ios::end);
  const size_t bytes = (size_t)f.tellg();
  f.seekg(0);
  if (bytes != expect * 4) return false;
  v.resize(expect);
  f.read((char*)v.data(), (std::streamsize)bytes);
  return (bool)f;
}

static void save_f32(const std::string& path, const std::vector<float>& v) {
  std::ofstream f(path, std::ios::binary);
  f.write((const char*)v.data(), (std::streamsize)(v.size() * 4));
}

static bool exists(const std::string& p) {
  std::ifstream f(p);
  return (bool)f;
}

// One stage of the last forward as image 0's fp32 NCHW tensor: int8 NHWC
// stages dequantised with their site scale, fp32 stages copied.
static int stage_image0(dlq_resnet18* m, bool fp32, const char* name, int C, int H, float scale, std::vector<float>& f) {
  const size_t n = (size_t)C * H * H;  // image 0 only, as the reference (N=1)
  size_t bytes = 0;
  void* tmp = nullptr;
  f.assign(n, 0.f);
  if (fp32) {
    CHECK_DLQ(dlq_resnet18_stage_f32(m, name, nullptr, 0, &bytes, nullptr));
    CHECK_HIP(hipMalloc(&tmp, bytes));
    CHECK_DLQ(dlq_resnet18_stage_f32(m, name, tmp, bytes, &bytes, nullptr));
    CHECK_HIP(hipMemcpy(f.data(), tmp, n * 4, hipMemcpyDeviceToHost));
  } else {
    std::vector<int8_t> q(n);
    CHECK_DLQ(dlq_resnet18_stage(m, name, nullptr, 0, &bytes, nullptr));
    CHECK_HIP(hipMalloc(&tmp, bytes));
    CHECK_DLQ(dlq_resnet18_stage(m, name, tmp, bytes, &bytes, nullptr));
    CHECK_HIP(hipMemcpy(q.data(), tmp, n, hipMemcpyDeviceToHost));
    for (int h = 0; h < H; ++h)  // NHWC int8 -> NCHW fp32
      for (int w = 0; w < H; ++w)
        for (int c = 0; c < C; ++c) f[((size_t)c * H + h) * H + w] = (float)q[((size_t)h * H + w) * C + c] * scale;
  }
  CHECK_HIP(hipFree(tmp));
  return 0;
}

int main(int argc, char** argv) {
  std::string mani, input, scales, dump, save_scales;
  int batch = 1, iters = 0, warmup = 0;
  bool fp32 = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--manifest" && i + 1 < argc) mani = argv[++i];
    else if (a == "--input" && i + 1 < argc) input = argv[++i];
    else if (a == "--scales" && i + 1 < argc) scales = argv[++i];
    else if (a == "--save_scales" && i + 1 < argc) save_scales = argv[++i];
    else if (a == "--dump_dir" && i + 1 < argc) dump = argv[++i];
    else if (a == "--fp32") fp32 = true;
    else if (a == "--batch" && i + 1 < argc) batch = std::atoi(argv[++i]);
    else if (a == "--iters" && i + 1 < argc) iters = std::atoi(argv[++i]);
    else if (a == "--warmup" && i + 1 < argc) warmup = std::atoi(argv[++i]);
  }
  if (mani.empty() || input.empty() || batch <= 0) {
    usage();
    return 1;
  }
  const size_t img = 3 * 224 * 224;
  std::vector<float> x;
  if (!load_f32(input, x, img)) {
    std::fprintf(stderr, "open/size fail: %s\n", input.c_str());
    return 1;
  }
  dlq_resnet18* m = nullptr;
  CHECK_DLQ(dlq_resnet18_create(&m));
  CHECK_DLQ(dlq_resnet18_load_manifest(m, mani.c_str()));

  float *dx = nullptr, *dlog = nullptr;
  CHECK_HIP(hipMalloc(&dx, img * 4 * batch));
  CHECK_HIP(hipMalloc(&dlog, (size_t)batch * 1000 * 4));
  for (int b = 0; b < batch; ++b)
    CHECK_HIP(hipMemcpy(dx + (size_t)b * img, x.data(), img * 4, hipMemcpyHostToDevice));

  if (!fp32) {
    if (scales.empty() && exists(mani + "/scales.txt")) scales = mani + "/scales.txt";
    if (!scales.empty()) {
      CHECK_DLQ(dlq_resnet18_load_scales(m, scales.c_str()));
    } else {
      CHECK_DLQ(dlq_resnet18_calibrate(m, dx, 1, 127.0f, nullptr));
      std::fprintf(stderr, "[E2E] no --scales and no %s/scales.txt: calibrated the int8 activation scales on the input\n",
                   mani.c_str());
    }
    if (!save_scales.empty()) CHECK_DLQ(dlq_resnet18_save_scales(m, save_scales.c_str()));
    CHECK_DLQ(dlq_resnet18_set_keep_stages(m, dump.empty() ? 0 : 1));
    CHECK_DLQ(dlq_resnet18_prepare(m, batch, nullptr));
    CHECK_DLQ(dlq_resnet18_forward(m, dx, batch, dlog, nullptr));
  } else {
    CHECK_DLQ(dlq_resnet18_forward_f32(m, dx, batch, dlog, nullptr));
  }
  CHECK_HIP(hipDeviceSynchronize());

  std::vector<float> logits(1000);
  CHECK_HIP(hipMemcpy(logits.data(), dlog, 4000, hipMemcpyDeviceToHost));
  int top = -1;
  float best = -1e30f;
  for (int i = 0; i < 1000; ++i)
    if (logits[i] > best) { best = logits[i]; top = i; }
  std::printf("[E2E] top-1 class index = %d, logit=%g\n", top, best);  // infer_e2e.cu:436-438

  if (!dump.empty()) {
    std::error_code ec;
    std::filesystem::create_directories(dump, ec);
    if (ec) {
      std::fprintf(stderr, "cannot create %s: %s\n", dump.c_str(), ec.message().c_str());
      return 2;
    }
    std::map<std::string, float> sc;
    if (!fp32) {  // dequantisation scales of the int8 stages
      const std::string tmp = dump + "/.scales.txt";
      CHECK_DLQ(dlq_resnet18_save_scales(m, tmp.c_str()));
      std::ifstream f(tmp);
      std::string line, site;
      float s;
      while (std::getline(f, line)) {
        std::istringstream ss(line);
        if (line[0] != '#' && (ss >> site >> s)) sc[site] = s;
      }
      std::filesystem::remove(tmp, ec);
    }
    struct St { const char* name; const char* site; int C, H; };
    const St st[] = {{"stem_pool", "conv1", 64, 56},        {"layer1", "layer1.1.conv2", 64, 56},
                     {"layer2", "layer2.1.conv2", 128, 28}, {"layer3", "layer3.1.conv2", 256, 14},
                     {"layer4", "layer4.1.conv2", 512, 7},  {"gap", "gap", 512, 1}};
    for (const auto& s : st) {
      std::vector<float> f;
      if (int rc = stage_image0(m, fp32, s.name, s.C, s.H, fp32 ? 1.f : sc[s.site], f)) return rc;
      save_f32(dump + "/" + s.name + ".bin", f);
    }
    save_f32(dump + "/logits.bin", logits);
  }

  if (iters > 0) {
    if (fp32) {
      std::fprintf(stderr, "--iters times the int8 engine; not available with --fp32\n");
      return 1;
    }
    hipEvent_t a, b;
    CHECK_HIP(hipEventCreate(&a));
    CHECK_HIP(hipEventCreate(&b));
    for (int i = 0; i < warmup; ++i) CHECK_DLQ(dlq_resnet18_forward(m, dx, batch, dlog, nullptr));
    CHECK_HIP(hipEventRecord(a, nullptr));
    for (int i = 0; i < iters; ++i) CHECK_DLQ(dlq_resnet18_forward(m, dx, batch, dlog, nullptr));
    CHECK_HIP(hipEventRecord(b, nullptr));
    CHECK_HIP(hipEventSynchronize(b));
    float ms = 0;
    CHECK_HIP(hipEventElapsedTime(&ms, a, b));
    std::printf("[E2E] batch=%d iters=%d  %.4f ms/forward  %.1f images/s\n", batch, iters, ms / iters,
                batch * iters * 1000.0 / ms);
  }
  (void)hipFree(dx);
  (void)hipFree(dlog);
  dlq_resnet18_destroy(m);
  return 0;
}
