// (Opt-in, VFD_STEM_CONV=1: as written these run slower than MIOpen — pose stem forward 613 us vs
// 286, weight gradient 502 vs 252 — because every 4 MFMAs wait on a per-lane gathered, bounds-
// checked operand; an LDS-staged input patch is the fix.  Kept with its parity test.)
//
// The ResNet encoders' stem: conv1 = Conv2d(C, 64, 7, stride 2, padding 3, no bias) applied to
// the normalised image (x - 0.45) / 0.225 (packnet ResnetEncoder, used at fusion_depthnet.py:24 /
// fusion_posenet.py:22; C = 3 for the depth net, 6 = two frames for the pose net).  MIOpen runs the
// pose stem at ~58 TF forward (238 us) and ~233 us for its weight gradient; here both are fp32
// MFMA implicit GEMMs (v_mfma_f32_16x16x4_f32) that read the raw image and normalise on load
// (padding stays zero in the normalised space, as in the reference):
//
//   forward  y[o][p] = sum_k A[p][k] W[o][k]        M = 16 consecutive output columns, N = 64,
//            K = C*49 (k = c*49 + ky*7 + kx, padded to a multiple of 4); W^T in LDS, the A operand
//            gathered per lane (stride-2 columns: a 16-lane group reads a 128-B span)
//   wgrad    dW[o][k] = sum_p dy[o][p] A[p][k]      M = 64, N = 16-wide k tiles (a block's share
//            of the k tiles), K = output pixels (4 per step); per-block partials summed by the caller
#include "vfd_common.h"

namespace vfd {

typedef float f32x4s __attribute__((ext_vector_type(4)));

constexpr int SC_THREADS = 256;
constexpr int SC_O = 64;

__device__ __forceinline__ f32x4s mfma16s(float a, float b, f32x4s c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// normalised input value at (n, c, iy, ix) (zero outside the image): the reference's
// (image - 0.45) / 0.225, evaluated as ATen's GPU kernels do (multiply by the fp32 reciprocal)
__device__ __forceinline__ float sc_in(const float* __restrict__ img, int C, int H, int W, int n, int c, int iy, int ix) {
  const bool ok = iy >= 0 && iy < H && ix >= 0 && ix < W;
  const float v = img[(((size_t)n * C + c) * H + (ok ? iy : 0)) * W + (ok ? ix : 0)];
  return ok ? (v - 0.45f) * (1.0f / 0.225f) : 0.f;
}

constexpr int SC_OH = 32;                        // output channels per block (grid.y = 64 / 32)
constexpr int SC_WH = SC_OH + 4;                 // LDS row stride of the block's W^T half
template <int C>
__global__ __launch_bounds__(SC_THREADS) void stem_fwd_k(const float* __restrict__ img, const float* __restrict__ w,
                                                         float* __restrict__ y, int N, int H, int W, int Ho, int Wo) {
  constexpr int K = C * 49, KS = (K + 3) / 4;    // k-steps of 4
  constexpr int NT = SC_OH / 16;
  __shared__ float wt[KS * 4 * SC_WH];           // W^T [k][o - o0], zero rows past K
  __shared__ int ktab[KS * 4];                   // k -> c << 16 | ky << 8 | kx
  const int o0 = blockIdx.y * SC_OH;
  for (int i = threadIdx.x; i < KS * 4 * SC_OH; i += SC_THREADS) {
    const int k = i / SC_OH, o = i - k * SC_OH;
    wt[k * SC_WH + o] = k < K ? w[(o0 + o) * K + k] : 0.f;
  }
  for (int k = threadIdx.x; k < KS * 4; k += SC_THREADS) {
    const int kk = k < K ? k : 0;
    const int c = kk / 49, r = kk - c * 49;
    ktab[k] = (c << 16) | ((r / 7) << 8) | (r % 7);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  const int tpr = Wo / 16;
  const long long ntile = (long long)N * Ho * tpr;
  const long long nw = (long long)gridDim.x * (SC_THREADS / 64);
  for (long long tile = (long long)blockIdx.x * (SC_THREADS / 64) + (threadIdx.x >> 6); tile < ntile; tile += nw) {
    const int x0 = (int)(tile % tpr) * 16;
    const int yo = (int)((tile / tpr) % Ho), n = (int)(tile / ((long long)tpr * Ho));
    f32x4s acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4s{0.f, 0.f, 0.f, 0.f};
    const int iy0 = 2 * yo - 3, ix0 = 2 * (x0 + li) - 3;      // this lane's A row (output column x0 + li)
    // A operand of k-step s (k = 4 s + lk), fetched two steps ahead of its MFMAs
    auto load_a = [&](int s) {
      const int k = 4 * s + lk;
      const int e = ktab[k < KS * 4 ? k : 0];
      const float a = sc_in(img, C, H, W, n, e >> 16, iy0 + ((e >> 8) & 255), ix0 + (e & 255));
      return k < K ? a : 0.f;
    };
    float a0 = load_a(0), a1 = load_a(1);
#pragma unroll 1
    for (int s = 0; s < KS; ++s) {
      const float a2 = load_a(s + 2);
      const int k = 4 * s + lk;
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma16s(a0, wt[k * SC_WH + 16 * t + li], acc[t]);
      a0 = a1;
      a1 = a2;
    }
    // D[i][j]: output column x0 + 4 lk + r, channel o0 + 16 t + li: one 16-B store per lane and tile
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float* dst = y + (((size_t)n * SC_O + o0 + 16 * t + li) * Ho + yo) * Wo + x0 + 4 * lk;
      *reinterpret_cast<float4*>(dst) = make_float4(acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
    }
  }
}

// weight gradient: block (pixel range g, k-tile group kg) accumulates dW[64][16 * SC_KT k-columns]
// over its pixels (4 per MFMA step, waves interleaved), combines its waves in LDS in wave order and
// writes partial[g][kg tiles][64][16]
constexpr int SC_KT = 4;                         // k tiles (of 16) per block
template <int C>
__global__ __launch_bounds__(SC_THREADS) void stem_wgrad_k(const float* __restrict__ img, const float* __restrict__ dy,
                                                           float* __restrict__ partial, int N, int H, int W, int Ho,
                                                           int Wo, long long groups_per_block, int nkg) {
  constexpr int K = C * 49;
  __shared__ float red[SC_KT * 16 * SC_O];
  const int kg = blockIdx.x % nkg;
  const long long gb = blockIdx.x / nkg;
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4, wv = threadIdx.x >> 6;
  const int gpr = Wo / 4;
  const long long ngroup = (long long)N * Ho * gpr;
  const long long g0 = gb * groups_per_block;
  const long long g1 = g0 + groups_per_block < ngroup ? g0 + groups_per_block : ngroup;
  // this lane's B column per k tile: k = 16 (SC_KT kg + b) + li -> (c, ky, kx)
  int kc[SC_KT], kyy[SC_KT], kxx[SC_KT];
  bool kin[SC_KT];
#pragma unroll
  for (int b = 0; b < SC_KT; ++b) {
    const int k = 16 * (SC_KT * kg + b) + li;
    kin[b] = k < K;
    const int kk = kin[b] ? k : 0;
    kc[b] = kk / 49;
    const int r = kk - kc[b] * 49;
    kyy[b] = r / 7;
    kxx[b] = r % 7;
  }
  f32x4s acc[4][SC_KT];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < SC_KT; ++b) acc[a][b] = f32x4s{0.f, 0.f, 0.f, 0.f};
  for (long long g = g0 + wv; g < g1; g += SC_THREADS / 64) {
    const int x0 = (int)(g % gpr) * 4;
    const int yo = (int)((g / gpr) % Ho), n = (int)(g / ((long long)gpr * Ho));
    // A[i = o][k = pixel x0 + lk] = dy[o][yo][x0 + lk]
    float av[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) av[a] = dy[(((size_t)n * SC_O + 16 * a + li) * Ho + yo) * Wo + x0 + lk];
    // B[k = pixel][j = k column] = normalised input under output (yo, x0 + lk) at tap (c, ky, kx)
    const int iy0 = 2 * yo - 3, ix0 = 2 * (x0 + lk) - 3;
    float bv[SC_KT];
#pragma unroll
    for (int b = 0; b < SC_KT; ++b) {
      const float v = sc_in(img, C, H, W, n, kc[b], iy0 + kyy[b], ix0 + kxx[b]);
      bv[b] = kin[b] ? v : 0.f;
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < SC_KT; ++b) acc[a][b] = mfma16s(av[a], bv[b], acc[a][b]);
  }
  // D[i = o][j = k column]: lane holds o = 16 a + 4 lk + r, column 16 b + li
  for (int w = 0; w < SC_THREADS / 64; ++w) {
    if (wv == w) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < SC_KT; ++b)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* p = red + (b * SC_O + 16 * a + 4 * lk + r) * 16 + li;
            *p = (w == 0 ? 0.f : *p) + acc[a][b][r];
          }
    }
    __syncthreads();
  }
  float* dst = partial + ((size_t)gb * nkg + kg) * SC_KT * SC_O * 16;
  for (int i = threadIdx.x; i < SC_KT * SC_O * 16; i += SC_THREADS) dst[i] = red[i];
}

static int sc_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 256;
  return cus;
}

}  // namespace vfd

using namespace vfd;

extern "C" {

int vfd_stem_conv_supported(int N, int C, int H, int W, int O) {
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  return N > 0 && (C == 3 || C == 6) && O == SC_O && H > 0 && W > 0 && Wo % 16 == 0 &&
         (long long)N * SC_O * Ho * Wo < (1LL << 31) && (long long)N * C * H * W < (1LL << 31);
}

int vfd_stem_conv_ktiles(int C) { return (C * 49 + 15) / 16; }

int vfd_stem_conv_wgrad_groups(void) { return sc_cus(); }

int vfd_stem_conv_fwd(const float* img, const float* w, float* y, int N, int C, int H, int W, void* stream) {
  VFD_REQUIRE(vfd_stem_conv_supported(N, C, H, W, SC_O), "stem_conv: unsupported shape (C in {3, 6}, 64 outputs, W/2 %% 16 == 0)");
  VFD_REQUIRE(img && w && y && ((uintptr_t)y & 15) == 0, "stem_conv_fwd: bad argument");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_STEM_CONV, s);
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const long long ntile = (long long)N * Ho * (Wo / 16);
  const long long need = (ntile + 3) / 4, most = (long long)sc_cus() * 3;
  const dim3 grid((unsigned)(need < most ? need : most), SC_O / SC_OH);
  if (C == 3) stem_fwd_k<3><<<grid, SC_THREADS, 0, s>>>(img, w, y, N, H, W, Ho, Wo);
  else stem_fwd_k<6><<<grid, SC_THREADS, 0, s>>>(img, w, y, N, H, W, Ho, Wo);
  return fail_launch("stem_conv_fwd");
}

// partial: [vfd_stem_conv_wgrad_groups()][ceil(ktiles / 4)][4][64][16] (k tiles past the last are zero)
int vfd_stem_conv_wgrad(const float* img, const float* dy, float* partial, int N, int C, int H, int W, void* stream) {
  VFD_REQUIRE(vfd_stem_conv_supported(N, C, H, W, SC_O), "stem_conv: unsupported shape");
  VFD_REQUIRE(img && dy && partial, "stem_conv_wgrad: bad argument");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_STEM_CONV, s);
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int nkg = (vfd_stem_conv_ktiles(C) + SC_KT - 1) / SC_KT;
  const int ng = vfd_stem_conv_wgrad_groups();
  const long long ngroup = (long long)N * Ho * (Wo / 4);
  const long long per = (ngroup + ng - 1) / ng;
  const unsigned grid = (unsigned)(ng * nkg);
  if (C == 3) stem_wgrad_k<3><<<grid, SC_THREADS, 0, s>>>(img, dy, partial, N, H, W, Ho, Wo, per, nkg);
  else stem_wgrad_k<6><<<grid, SC_THREADS, 0, s>>>(img, dy, partial, N, H, W, Ho, Wo, per, nkg);
  return fail_launch("stem_conv_wgrad");
}

}  // extern "C"
