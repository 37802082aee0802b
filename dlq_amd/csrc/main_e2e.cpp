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
// Additions: --scales FILE (the int8 activation scales; required),
// --batch B (replicate the image), --iters/--warmup (hipEvent timing).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
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
      "dlq_e2e --manifest <dir> --input <input.bin> --scales <scales.txt> [--dump_dir <dir>]\n"
      "        [--batch B] [--iters K] [--warmup W]\n");
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

int main(int argc, char** argv) {
  std::string mani, input, scales, dump;
  int batch = 1, iters = 0, warmup = 0;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--manifest" && i + 1 < argc) mani = argv[++i];
    else if (a == "--input" && i + 1 < argc) input = argv[++i];
    else if (a == "--scales" && i + 1 < argc) scales = argv[++i];
    else if (a == "--dump_dir" && i + 1 < argc) dump = argv[++i];
    else if (a == "--batch" && i + 1 < argc) batch = std::atoi(argv[++i]);
    else if (a == "--iters" && i + 1 < argc) iters = std::atoi(argv[++i]);
    else if (a == "--warmup" && i + 1 < argc) warmup = std::atoi(argv[++i]);
  }
  if (mani.empty() || input.empty() || scales.empty() || batch <= 0) {
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
  CHECK_DLQ(dlq_resnet18_load_scales(m, scales.c_str()));
  CHECK_DLQ(dlq_resnet18_set_keep_stages(m, dump.empty() ? 0 : 1));
  CHECK_DLQ(dlq_resnet18_prepare(m, batch, nullptr));

  float *dx = nullptr, *dlog = nullptr;
  CHECK_HIP(hipMalloc(&dx, img * 4 * batch));
  CHECK_HIP(hipMalloc(&dlog, (size_t)batch * 1000 * 4));
  for (int b = 0; b < batch; ++b)
    CHECK_HIP(hipMemcpy(dx + (size_t)b * img, x.data(), img * 4, hipMemcpyHostToDevice));
  CHECK_DLQ(dlq_resnet18_forward(m, dx, batch, dlog, nullptr));
  CHECK_HIP(hipDeviceSynchronize());

  std::vector<float> logits(1000);
  CHECK_HIP(hipMemcpy(logits.data(), dlog, 4000, hipMemcpyDeviceToHost));
  int top = -1;
  float best = -1e30f;
  for (int i = 0; i < 1000; ++i)
    if (logits[i] > best) { best = logits[i]; top = i; }
  std::printf("[E2E] top-1 class index = %d, logit=%f\n", top, best);

  if (!dump.empty()) {
    std::string cmd = "mkdir -p '" + dump + "'";
    if (std::system(cmd.c_str()) != 0) std::fprintf(stderr, "mkdir failed: %s\n", dump.c_str());
    std::map<std::string, float> sc;
    {
      std::ifstream f(scales);
      std::string site; float s;
      std::string line;
      while (std::getline(f, line)) {
        std::istringstream ss(line);
        if (ss >> site >> s) sc[site] = s;
      }
    }
    struct St { const char* name; const char* site; int C, H; };
    const St st[] = {{"stem_pool", "conv1", 64, 56},        {"layer1", "layer1.1.conv2", 64, 56},
                     {"layer2", "layer2.1.conv2", 128, 28}, {"layer3", "layer3.1.conv2", 256, 14},
                     {"layer4", "layer4.1.conv2", 512, 7}};
    for (const auto& s : st) {
      const size_t n = (size_t)s.C * s.H * s.H;  // image 0 only, as the reference (N=1)
      std::vector<int8_t> q(n);
      int8_t* tmp = nullptr;
      size_t bytes = 0;
      CHECK_DLQ(dlq_resnet18_stage(m, s.name, nullptr, 0, &bytes, nullptr));
      CHECK_HIP(hipMalloc(&tmp, bytes));
      CHECK_DLQ(dlq_resnet18_stage(m, s.name, tmp, bytes, &bytes, nullptr));
      CHECK_HIP(hipMemcpy(q.data(), tmp, n, hipMemcpyDeviceToHost));
      CHECK_HIP(hipFree(tmp));
      std::vector<float> f(n);  // NHWC int8 -> NCHW fp32
      for (int h = 0; h < s.H; ++h)
        for (int w = 0; w < s.H; ++w)
          for (int c = 0; c < s.C; ++c)
            f[((size_t)c * s.H + h) * s.H + w] = (float)q[((size_t)h * s.H + w) * s.C + c] * sc[s.site];
      save_f32(dump + "/" + s.name + ".bin", f);
    }
    {
      std::vector<int8_t> g(512);
      int8_t* tmp = nullptr;
      size_t bytes = 0;
      CHECK_DLQ(dlq_resnet18_stage(m, "gap", nullptr, 0, &bytes, nullptr));
      CHECK_HIP(hipMalloc(&tmp, bytes));
      CHECK_DLQ(dlq_resnet18_stage(m, "gap", tmp, bytes, &bytes, nullptr));
      CHECK_HIP(hipMemcpy(g.data(), tmp, 512, hipMemcpyDeviceToHost));
      CHECK_HIP(hipFree(tmp));
      std::vector<float> f(512);
      for (int c = 0; c < 512; ++c) f[c] = (float)g[c] * sc["gap"];
      save_f32(dump + "/gap.bin", f);
    }
    save_f32(dump + "/logits.bin", logits);
  }

  if (iters > 0) {
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
