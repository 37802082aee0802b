// conv3x3.hip -- stride-1 3x3 int8 conv (the 12 "layerX.Y.conv{1,2}" launches
// of ResNet-18 that keep the resolution) with an LDS-resident input patch.
//
// Replaces im2col_nchw + sgemm_tiled + bn/add/relu (RK/kernels/im2col.cu:5-58,
// sgemm_tiled.cu:5-46; launched from RK/runtime/infer_e2e.cu:102-136,156-203)
// for these shapes.  Where the v1 implicit-GEMM kernel re-reads every input
// pixel once per tap (9x for a 3x3 conv), this kernel stages the input rows a
// pixel tile needs (the "patch": the tile's rows plus a 1-row halo, one
// 64-channel chunk) into LDS once and forms all nine taps from it.
//
// Work item = (256 consecutive output pixels in (n, oh, ow) order) x (64 output
// channels).  Persistent grid (one NWAVE-wave workgroup per CU); each
// workgroup walks its items; a stage = one 64-channel input chunk of one item:
//   patch (LDS-DMA, XOR-swizzled 64-byte pixel rows) + the 64x9x64-byte weight
//   block of that chunk (LDS-DMA, verbatim copy of the packed image) [+ the
//   item's residual tile on its last chunk].
// Stages are double buffered: stage s+1's LDS-DMA is in flight while stage
// s's 9 taps x 2 k-halves of v_mfma_i32_32x32x32_i8 run.  Each wave owns 64 oc
// x (256/NWAVE) pixels.  With 8 waves, two per SIMD, one wave's VALU epilogue
// overlaps its partner's MFMAs.  Halo rows and columns are never loaded: taps
// that fall outside the image read 64 zero bytes in LDS instead.  The
// epilogue is the fused dequant*BN, residual, ReLU, requant sequence of the
// v1 kernel; int8 results are staged in LDS per wave and stored as whole
// 64-byte pixel rows.
#include "device_common.h"

namespace dlq {

__device__ __attribute__((aligned(64))) int8_t g_trash[1024];  // sink for masked-off epilogue lanes

namespace {

template <int W, int C, int TP>
struct PatchCfg {
  static constexpr int H = W;
  static constexpr int ROWS = (TP + W - 1) / W + 1;            // output rows a tile can touch
  static constexpr int IMGS = (TP + H * W - 1) / (H * W) + 1;  // images a tile can touch
  static constexpr int SLOTS = ROWS + 2 * IMGS;                // input rows (per image: rows + 2 halo)
  static constexpr int UNITS = SLOTS * W * 4;                  // 16-byte units (no halo columns)
  static constexpr int PIECES = (UNITS + 63) / 64;             // 1 KiB LDS-DMA wave pieces
  static constexpr int PBYTES = PIECES * 1024;
  static constexpr int NCH = C / 64;
  static constexpr bool RESIDENT = (NCH == 1);  // single chunk: weights stay in LDS
};

constexpr int TOC = 64;
constexpr int TP = 256;
constexpr int WBYTES = TOC * 9 * 64;  // one chunk's weight block (packed image, verbatim)
constexpr int WPIECES = WBYTES / 1024;

// OUT: 0 = int8 (fused epilogue), 2 = int32 accumulators.
template <int W, int C, int NWAVE, int OUT, bool RES>
__global__ __launch_bounds__(NWAVE * 64, 1) void conv3x3s1_kernel(ConvArgs a) {
  using G = PatchCfg<W, C, TP>;
  constexpr int H = W, NCH = G::NCH, NTH = NWAVE * 64;
  constexpr int PXW = TP / NWAVE;  // pixels per wave
  constexpr int FN = PXW / 32;     // 32-pixel MFMA tiles per wave
  constexpr int NST = PXW / 16;    // epilogue 16-B stores per lane (= per wave instruction count)
  static_assert(FN >= 1 && PXW % 32 == 0, "wave tile");
  constexpr int NWB = G::RESIDENT ? 1 : 2;
  // residual tiles (2 when the next item's tile is prefetched during this
  // item's only stage); they double as the per-wave output staging area.
  constexpr int NSB = RES ? (NCH == 1 ? 2 : 1) : 1;
  constexpr int SBYTES = TP * TOC;
  constexpr int OFF_W = 2 * G::PBYTES;
  constexpr int OFF_S = OFF_W + NWB * WBYTES;
  constexpr int OFF_AB = OFF_S + NSB * SBYTES;
  constexpr int OFF_Z = OFF_AB + 2 * 512 * 4;  // 64 zero bytes: the conv's zero padding
  constexpr int LDS_TOTAL = OFF_Z + 64;
  static_assert(LDS_TOTAL <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) int8_t lds[LDS_TOTAL];
  float* s_alpha = (float*)(lds + OFF_AB);
  float* s_beta = s_alpha + 512;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const int n_ot = a.OCp / TOC;
  const int NI = n_ot * ((a.P + TP - 1) / TP);
  const int Gd = gridDim.x, b = blockIdx.x;
  const int nstages = ((NI - b + Gd - 1) / Gd) * NCH;

  if constexpr (OUT == 0) {
    for (int i = tid; i < a.OCp; i += NTH) {
      s_alpha[i] = a.alpha[i];
      s_beta[i] = a.beta[i];
    }
  }
  if (tid < 16) ((int*)(lds + OFF_Z))[tid] = 0;
  __syncthreads();  // before any LDS-DMA is in flight (its vmcnt(0) would drain it)
  if constexpr (G::RESIDENT) {
    for (int pc = wave; pc < WPIECES; pc += NWAVE) glds16(a.w + pc * 1024 + lane * 16, lds + OFF_W + pc * 1024);
  }

  struct Tile {
    int ot, p0, pend, n0, oh0, cnt0, units;
  };
  auto tile_of = [&](int it) {
    Tile t;
    t.ot = it % n_ot;
    t.p0 = (it / n_ot) * TP;
    t.pend = min(t.p0 + TP, a.P);
    const int R0 = t.p0 / W, R1 = (t.pend - 1) / W;
    t.n0 = R0 / H;
    t.oh0 = R0 - t.n0 * H;
    const int n1 = R1 / H;
    t.cnt0 = ((n1 == t.n0) ? (R1 - R0) : (H - 1 - t.oh0)) + 3;
    const int slots = (n1 == t.n0) ? t.cnt0 : t.cnt0 + (n1 - t.n0 - 1) * (H + 2) + (R1 - n1 * H) + 3;
    t.units = slots * W * 4;
    return t;
  };

  // LDS-DMA of stage s: the patch rows the tile needs (64-byte pixel rows,
  // chunk-swizzled by row), the chunk's weight block, and on the item's last
  // chunk its residual tile.  Slot rows of the 1-row halo outside the image
  // are not fetched (their LDS is never read).
  auto issue = [&](int s) {
    const int li = s / NCH, ch = s - li * NCH;
    const Tile t = tile_of(b + li * Gd);
    int8_t* pb = lds + (s & 1) * G::PBYTES;
    const int npieces = (t.units + 63) >> 6;
    for (int pc = wave; pc < npieces; pc += NWAVE) {
      const int u = pc * 64 + lane;
      const int q = u >> 2, pch = u & 3;
      const int slot = q / W, col = q - slot * W;
      const int lc = pch ^ ((q >> 2) & 3);
      int n, ih;
      if (slot < t.cnt0) {
        n = t.n0;
        ih = t.oh0 - 1 + slot;
      } else {
        const int s2 = slot - t.cnt0;
        n = t.n0 + 1 + s2 / (H + 2);
        ih = s2 % (H + 2) - 1;
      }
      const bool ok = u < t.units && (unsigned)ih < (unsigned)H;
      const int8_t* src = a.x + (ok ? ((size_t)(n * H + ih) * W + col) * C + ch * 64 + lc * 16 : 0);
      glds16(src, pb + pc * 1024);
    }
    if constexpr (!G::RESIDENT) {
      const int8_t* wsrc = a.w + ((size_t)ch * n_ot + t.ot) * WBYTES;
      int8_t* wb = lds + OFF_W + (s & 1) * WBYTES;
      for (int pc = wave; pc < WPIECES; pc += NWAVE) glds16(wsrc + pc * 1024 + lane * 16, wb + pc * 1024);
    }
    if constexpr (RES) {
      if (ch == NCH - 1) {  // the item's residual tile [256 px][64 oc], chunk-swizzled by px
        int8_t* rb = lds + OFF_S + (NSB == 2 ? (li & 1) : 0) * SBYTES;
        for (int pc = wave; pc < SBYTES / 1024; pc += NWAVE) {
          const int u = pc * 64 + lane, px = u >> 2, pch = u & 3;
          const int lc = pch ^ ((px >> 2) & 3);
          const int p = min(t.p0 + px, a.P - 1);
          glds16(a.res + (size_t)p * a.OC + t.ot * 64 + lc * 16, rb + pc * 1024);
        }
      }
    }
  };

  // Lane-constant A (weight) fragment offsets: row oc_local, chunk 2kk+lh swizzled.
  int a_off[2][2];
#pragma unroll
  for (int fm = 0; fm < 2; ++fm)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ol = fm * 32 + lr;
      a_off[fm][kk] = ol * 576 + (((2 * kk + lh) ^ ((ol >> 2) & 3)) << 4);
    }

  v16i acc[2][FN];
  int rowbase[FN];      // patch row of tap (kh=0, kw=1) for the lane's pixel of tile fn
  unsigned vmask[FN];   // bit kh*3+kw: tap inside the image
  Tile cur{};

  issue(0);
  for (int s = 0; s < nstages; ++s) {
    const int li = s / NCH, ch = s - li * NCH;
    // Stage s's LDS-DMA must have landed; the previous item's NST epilogue
    // stores (issued after it, so the NST youngest VM ops) may stay in
    // flight.  Raw s_barrier: __syncthreads() would add a vmcnt(0).  The
    // waits are builtins (not inline asm) so hipcc's waitcnt pass sees them.
    if (OUT == 0 && s > 0 && ch == 0)
      __builtin_amdgcn_s_waitcnt(0x0070 | NST);  // vmcnt(NST) expcnt(7) lgkmcnt(0)
    else
      __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) expcnt(7) lgkmcnt(0)
    __builtin_amdgcn_s_barrier();

    if (ch == 0) {  // new item: lane pixel bases, zero accumulators
      cur = tile_of(b + li * Gd);
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int p = cur.p0 + wave * PXW + fn * 32 + lr;
        int rbv = 0;
        unsigned m = 0;
        if (p < cur.pend) {
          const int n = p / (H * W), r = p - n * (H * W), oh = r / W, ow = r - oh * W;
          const int slot0 = (n == cur.n0) ? oh - cur.oh0 : cur.cnt0 + (n - cur.n0 - 1) * (H + 2) + oh;
          rbv = slot0 * W + ow;
#pragma unroll
          for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw)
              if ((unsigned)(oh + kh - 1) < (unsigned)H && (unsigned)(ow + kw - 1) < (unsigned)W)
                m |= 1u << (kh * 3 + kw);
        }
        rowbase[fn] = rbv;
        vmask[fn] = m;
      }
#pragma unroll
      for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) acc[fm][fn] = v16i{0};
    }

    // Epilogue operands are read from LDS BEFORE the next stage's LDS-DMA is
    // issued, as int vectors (a float-typed LDS read made hipcc drain vmcnt
    // first, exposing the prefetch latency).
    float4 e_al[2][4], e_be[2][4];
    int e_rq[2][FN][4];
    if constexpr (OUT == 0) {
      if (ch == NCH - 1) {
        const int8_t* rb = lds + OFF_S + (NSB == 2 ? (li & 1) : 0) * SBYTES;
#pragma unroll
        for (int fm = 0; fm < 2; ++fm)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int ol = fm * 32 + 8 * g + 4 * lh;
            const v4i al4 = *(const v4i*)(lds + OFF_AB + (cur.ot * 64 + ol) * 4);
            const v4i be4 = *(const v4i*)(lds + OFF_AB + 2048 + (cur.ot * 64 + ol) * 4);
            e_al[fm][g] = make_float4(__int_as_float(al4[0]), __int_as_float(al4[1]), __int_as_float(al4[2]),
                                      __int_as_float(al4[3]));
            e_be[fm][g] = make_float4(__int_as_float(be4[0]), __int_as_float(be4[1]), __int_as_float(be4[2]),
                                      __int_as_float(be4[3]));
#pragma unroll
            for (int fn = 0; fn < FN; ++fn) {
              const int px = wave * PXW + fn * 32 + lr;
              e_rq[fm][fn][g] = 0;
              if constexpr (RES)
                e_rq[fm][fn][g] = (*(const v4i*)(rb + px * 64 + (((ol >> 4) ^ ((px >> 2) & 3)) << 4)))[(ol >> 2) & 3];
            }
          }
      }
    }
    if (s + 1 < nstages && !DLQ_ABL(a, 2)) issue(s + 1);

    const int8_t* pb = lds + (s & 1) * G::PBYTES;
    const int8_t* wb = lds + OFF_W + (G::RESIDENT ? 0 : (s & 1)) * WBYTES;
    // 18 steps (9 taps x 2 k-halves); fragments of step i+1 are read while
    // step i's MFMAs run.
    auto load_step = [&](int st, v4i (&af)[2], v4i (&bf)[FN]) {
      const int tap = st >> 1, kk = st & 1, kh = tap / 3, kw = tap % 3;
#pragma unroll
      for (int fm = 0; fm < 2; ++fm) af[fm] = *(const v4i*)(wb + a_off[fm][kk] + tap * 64);
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int q = rowbase[fn] + kh * W + kw - 1;
        const int off = q * 64 + (((2 * kk + lh) ^ ((q >> 2) & 3)) << 4);
        bf[fn] = *(const v4i*)(lds + (((vmask[fn] >> tap) & 1) ? (int)(pb - lds) + off : OFF_Z));
      }
    };
    if (!DLQ_ABL(a, 1)) {
      v4i af0[2], bf0[FN], af1[2], bf1[FN];
      load_step(0, af0, bf0);
#pragma unroll
      for (int st = 0; st < 18; st += 2) {
        load_step(st + 1, af1, bf1);
#pragma unroll
        for (int fm = 0; fm < 2; ++fm)
#pragma unroll
          for (int fn = 0; fn < FN; ++fn)
            acc[fm][fn] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af0[fm], bf0[fn], acc[fm][fn], 0, 0, 0);
        if (st + 2 < 18) load_step(st + 2, af0, bf0);
#pragma unroll
        for (int fm = 0; fm < 2; ++fm)
#pragma unroll
          for (int fn = 0; fn < FN; ++fn)
            acc[fm][fn] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af1[fm], bf1[fn], acc[fm][fn], 0, 0, 0);
      }
    }

    if (ch == NCH - 1) {  // ---- fused epilogue of the item ----
      if constexpr (OUT == 2) {
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const int p = cur.p0 + wave * PXW + fn * 32 + lr;
          if (p >= cur.pend) continue;
#pragma unroll
          for (int fm = 0; fm < 2; ++fm)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int oc = cur.ot * 64 + fm * 32 + 8 * g + 4 * lh;
              *(v4i*)((int*)a.y + (size_t)p * a.OC + oc) =
                  v4i{acc[fm][fn][4 * g], acc[fm][fn][4 * g + 1], acc[fm][fn][4 * g + 2], acc[fm][fn][4 * g + 3]};
            }
        }
      } else {
        // Requantise in the MFMA layout, stage this wave's PXW px x 64 oc int8
        // block in LDS, then store it as whole 64-byte pixel rows (16 B/lane).
        int8_t* sb = lds + OFF_S + (NSB == 2 ? (li & 1) : 0) * SBYTES + wave * (PXW * 64);
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const int pl = fn * 32 + lr;
#pragma unroll
          for (int fm = 0; fm < 2; ++fm)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int ol = fm * 32 + 8 * g + 4 * lh;
              const float4 al = e_al[fm][g], be = e_be[fm][g];
              const float alv[4] = {al.x, al.y, al.z, al.w};
              const float bev[4] = {be.x, be.y, be.z, be.w};
              const int rq = e_rq[fm][fn][g];
              float v[4];
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                v[j] = __builtin_fmaf((float)acc[fm][fn][4 * g + j], alv[j], bev[j]);
                if constexpr (RES) v[j] = __builtin_fmaf((float)(int)(signed char)(rq >> (8 * j)), a.s_res, v[j]);
              }
              const unsigned packed = quant4(v[0], v[1], v[2], v[3], a.relu ? 0.f : -127.f);
              *(unsigned*)(sb + pl * 64 + (((ol >> 4) ^ ((pl >> 2) & 3)) << 4) + ((ol >> 2) & 3) * 4) = packed;
            }
        }
        // The same wave reads its block back (LDS is in order per wave).
        // Exactly NST store instructions per wave, never skipped (the
        // loop-top vmcnt(NST) relies on it): lanes past the tile's end store
        // to g_trash.
#pragma unroll
        for (int r = 0; r < NST; ++r) {
          const int u = r * 64 + lane, pl = u >> 2, lc = u & 3;
          const v4i v = *(const v4i*)(sb + pl * 64 + ((lc ^ ((pl >> 2) & 3)) << 4));
          const int p = cur.p0 + wave * PXW + pl;
          const bool keep = p < cur.pend && (!DLQ_ABL(a, 4) || v[0] == 0x9e3779b9);
          v4i* dst = keep ? (v4i*)((int8_t*)a.y + (size_t)p * a.OC + cur.ot * 64 + lc * 16)
                          : (v4i*)(g_trash + lane * 16);
          *dst = v;
        }
      }
    }
  }
  wait_vm0();
}

constexpr int kWaves = 8;

template <int W, int C>
hipError_t launch_w(const ConvArgs& a, hipStream_t s, int ncu) {
  const int NI = (a.OCp / TOC) * ((a.P + TP - 1) / TP);
  const dim3 grid(NI < ncu ? NI : ncu), block(kWaves * 64);
  if (a.out_kind == 2)
    hipLaunchKernelGGL((conv3x3s1_kernel<W, C, kWaves, 2, false>), grid, block, 0, s, a);
  else if (a.res)
    hipLaunchKernelGGL((conv3x3s1_kernel<W, C, kWaves, 0, true>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((conv3x3s1_kernel<W, C, kWaves, 0, false>), grid, block, 0, s, a);
  return hipGetLastError();
}

int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

}  // namespace

bool conv3x3s1_supported(const ConvArgs& a) {
  if (!(a.kH == 3 && a.kW == 3 && a.sH == 1 && a.sW == 1 && a.pH == 1 && a.pW == 1)) return false;
  if (a.H != a.W || a.out_kind == 1 || a.OC % 64 || a.OCp % 64) return false;
  const bool shape = (a.W == 56 && a.C == 64) || (a.W == 28 && a.C == 128) || (a.W == 14 && a.C == 256) ||
                     (a.W == 7 && a.C == 512);
  if (!shape) return false;
  if (a.C == 64 && a.OCp != 64) return false;  // resident-weight variant needs one oc tile
  return true;
}

hipError_t launch_conv3x3s1(const ConvArgs& a, hipStream_t s) {
  const int ncu = num_cus();
  switch (a.W) {
    case 56: return launch_w<56, 64>(a, s, ncu);
    case 28: return launch_w<28, 128>(a, s, ncu);
    case 14: return launch_w<14, 256>(a, s, ncu);
    case 7: return launch_w<7, 512>(a, s, ncu);
  }
  return hipErrorInvalidValue;
}

}  // namespace dlq
