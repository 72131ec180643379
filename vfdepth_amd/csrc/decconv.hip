// The depth decoder's narrow 3x3 convolutions at the two finest levels (fusion_depthnet.py:97-145:
// upconv blocks with 16 / 32 channels at 192x320 and 384x640, reflect padding, stride 1) as fp32
// MFMA kernels on v_mfma_f32_16x16x4_f32.  MIOpen runs these narrow convs far below the matrix
// cores' rate (the 16 -> 16 conv at 384x640: ~170 us forward, ~440 us backward for 6.8 GFLOP each
// way); here each pass is an implicit GEMM whose N side is the 16-wide channel dimension:
//
//   forward   y[o][p]      = b[o] + sum_{c,tap} xp[c][p + tap] w[o][c][tap]      M = pixels (16 per
//             tile, consecutive x of one row), N = CO, K = 9 taps x CI
//   dgrad     dxp[c][P]    = sum_{o,tap} dy[o][P - tap] w[o][c][tap]            M = padded pixels,
//             N = CI, K = 9 x CO (dy = 0 outside the output grid: predicated loads)
//   wgrad     dw[o][c][tap] = sum_p dy[o][p] xp[c][p + tap]                      M = CO, N = CI per
//             tap, K = pixels (4 per MFMA step); per-block partials, summed by the caller
//
// Operand layouts (v_mfma_f32_16x16x4_f32): A[i][k] in lane i + 16 k, B[k][j] in lane j + 16 k,
// D[i][j] in lane j + 16 (i / 4), register i % 4.  The weights (B of the forward / data gradient)
// stay in registers for a wave's whole run of tiles; xp is read straight from L1/L2 (each element
// serves 9 taps of neighbouring k-steps).
#include "vfd_common.h"

namespace vfd {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int DK_THREADS = 256;

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// forward: a wave takes 16-pixel tiles (n, y, x0) in turn (grid-stride); W % 16 == 0
template <int CI, int CO>
__global__ __launch_bounds__(DK_THREADS) void dconv_fwd_k(const float* __restrict__ xp, const float* __restrict__ w,
                                                          const float* __restrict__ bias, float* __restrict__ y,
                                                          int N, int H, int W) {
  constexpr int NT = CO / 16, KQ = CI / 4;
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  const int wp = W + 2, hp = H + 2;
  // B[k][j] = w[16 t + j][4 q + k][tap]
  float bw[NT][9][KQ];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int q = 0; q < KQ; ++q) bw[t][tap][q] = w[((16 * t + li) * CI + 4 * q + lk) * 9 + tap];
  float bo[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) bo[t] = bias[16 * t + li];
  const int tpr = W / 16;
  const long long ntile = (long long)N * H * tpr;
  const long long nw = (long long)gridDim.x * (DK_THREADS / 64);
  for (long long tile = (long long)blockIdx.x * (DK_THREADS / 64) + (threadIdx.x >> 6); tile < ntile; tile += nw) {
    const int x0 = (int)(tile % tpr) * 16;
    const int yy = (int)((tile / tpr) % H), n = (int)(tile / ((long long)tpr * H));
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{bo[t], bo[t], bo[t], bo[t]};   // D column j = lane & 15
    const float* base = xp + (((size_t)n * CI + lk) * hp + yy) * wp + x0 + li;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap - 3 * ky;
      float a[KQ];
#pragma unroll
      for (int q = 0; q < KQ; ++q) a[q] = base[((size_t)(4 * q) * hp + ky) * wp + kx];   // A[i=li][k=lk]
#pragma unroll
      for (int q = 0; q < KQ; ++q)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16(a[q], bw[t][tap][q], acc[t]);
    }
    // D[i][j]: pixel x0 + 4 lk + r, channel 16 t + li: one 16-B store per lane and tile
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float* dst = y + (((size_t)n * CO + 16 * t + li) * H + yy) * W + x0 + 4 * lk;
      *reinterpret_cast<float4*>(dst) = make_float4(acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
    }
  }
}

// data gradient over the padded grid: tiles of 16 consecutive padded columns of one padded row
template <int CI, int CO>
__global__ __launch_bounds__(DK_THREADS) void dconv_dgrad_k(const float* __restrict__ dy, const float* __restrict__ w,
                                                            float* __restrict__ dxp, int N, int H, int W) {
  constexpr int NT = CI / 16, KQ = CO / 4;
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  const int wp = W + 2, hp = H + 2;
  // B[k][j] = w[4 q + k][16 t + j][tap]
  float bw[NT][9][KQ];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int q = 0; q < KQ; ++q) bw[t][tap][q] = w[((4 * q + lk) * CI + 16 * t + li) * 9 + tap];
  const int tpr = (wp + 15) / 16;
  const long long ntile = (long long)N * hp * tpr;
  const long long nw = (long long)gridDim.x * (DK_THREADS / 64);
  for (long long tile = (long long)blockIdx.x * (DK_THREADS / 64) + (threadIdx.x >> 6); tile < ntile; tile += nw) {
    const int X0 = (int)(tile % tpr) * 16;
    const int Y = (int)((tile / tpr) % hp), n = (int)(tile / ((long long)tpr * hp));
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int X = X0 + li;                                     // this lane's A row (padded column)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap - 3 * ky;
      const int yo = Y - ky, xo = X - kx;                      // output pixel reaching (Y, X) via tap
      const bool ok = yo >= 0 && yo < H && xo >= 0 && xo < W;
      const float* src = dy + (((size_t)n * CO + lk) * H + (ok ? yo : 0)) * W + (ok ? xo : 0);
      float a[KQ];
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        const float v = src[(size_t)(4 * q) * H * W];
        a[q] = ok ? v : 0.f;
      }
#pragma unroll
      for (int q = 0; q < KQ; ++q)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16(a[q], bw[t][tap][q], acc[t]);
    }
    // D[i][j]: padded column X0 + 4 lk + r, channel 16 t + li (columns past the padded width
    // dropped); two 8-B stores per lane (rows and X0 + 4 lk are even: wp = W + 2 is even)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float* dst = dxp + (((size_t)n * CI + 16 * t + li) * hp + Y) * wp + X0 + 4 * lk;
      const int left = wp - (X0 + 4 * lk);
      if (left >= 4) {
        *reinterpret_cast<float2*>(dst) = make_float2(acc[t][0], acc[t][1]);
        *reinterpret_cast<float2*>(dst + 2) = make_float2(acc[t][2], acc[t][3]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (r < left) dst[r] = acc[t][r];
      }
    }
  }
}

// weight gradient: a block walks strips of 64 consecutive output pixels of one row (W % 64 == 0).
// A strip's xp rows (3 x 66 columns x CI) and dy (CO x 64) are staged in LDS with coalesced loads
// (the MFMA operands are channel-strided: read straight from global memory every 16-lane group
// touches 16 planes); the next strip's loads are issued into registers before the current strip's
// MFMAs.  Each wave owns 16 of the strip's pixels (4 k-steps) and keeps the dW tiles of all taps
// in registers; waves are combined in LDS in wave order and the block writes
// partial[block][CO][CI][9].
constexpr int DW_S = 64;                        // pixels per strip
constexpr int DW_XS = DW_S + 3;                 // LDS row stride of the xp rows (66 used; bank spread)
constexpr int DW_GS = DW_S + 1;                 // LDS row stride of dy

template <int CI, int CO>
__global__ __launch_bounds__(DK_THREADS) void dconv_wgrad_k(const float* __restrict__ dy, const float* __restrict__ xp,
                                                            float* __restrict__ partial, int N, int H, int W,
                                                            long long strips_per_block) {
  constexpr int NO = CO / 16, NC = CI / 16;
  constexpr int XN = CI * 3 * (DW_S + 2), GN = CO * DW_S;           // staged floats
  constexpr int XPT = (XN + DK_THREADS - 1) / DK_THREADS, GPT = (GN + DK_THREADS - 1) / DK_THREADS;
  constexpr int LDS0 = CI * 3 * DW_XS + CO * DW_GS;
  constexpr int LDS = LDS0 > CO * CI * 9 ? LDS0 : CO * CI * 9;   // staging, then the wave reduction
  __shared__ float lds[LDS];
  float* xs = lds;
  float* gs = lds + CI * 3 * DW_XS;
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4, wv = threadIdx.x >> 6;
  const int wp = W + 2, hp = H + 2;
  const int spr = W / DW_S;
  const long long nstrip = (long long)N * H * spr;
  const long long s0 = (long long)blockIdx.x * strips_per_block;
  const long long s1 = s0 + strips_per_block < nstrip ? s0 + strips_per_block : nstrip;
  f32x4 acc[NO][9][NC];
#pragma unroll
  for (int a = 0; a < NO; ++a)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int b = 0; b < NC; ++b) acc[a][tap][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  float rx[XPT], rg[GPT];
  auto fetch = [&](long long s) {               // strip s -> registers (coalesced along columns)
    const int x0 = (int)(s % spr) * DW_S;
    const int yy = (int)((s / spr) % H), n = (int)(s / ((long long)spr * H));
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int k = threadIdx.x + i * DK_THREADS;
      const int kk = k < XN ? k : 0;
      const int col = kk % (DW_S + 2), row = kk / (DW_S + 2);            // row = c * 3 + ky
      const int c = row / 3, ky = row - 3 * c;
      rx[i] = xp[(((size_t)n * CI + c) * hp + yy + ky) * wp + x0 + col];
    }
#pragma unroll
    for (int i = 0; i < GPT; ++i) {
      const int k = threadIdx.x + i * DK_THREADS;
      const int kk = k < GN ? k : 0;
      const int col = kk % DW_S, o = kk / DW_S;
      rg[i] = dy[(((size_t)n * CO + o) * H + yy) * W + x0 + col];
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int k = threadIdx.x + i * DK_THREADS;
      if (k < XN) xs[(k / (DW_S + 2)) * DW_XS + k % (DW_S + 2)] = rx[i];
    }
#pragma unroll
    for (int i = 0; i < GPT; ++i) {
      const int k = threadIdx.x + i * DK_THREADS;
      if (k < GN) gs[(k / DW_S) * DW_GS + k % DW_S] = rg[i];
    }
  };
  if (s0 < s1) fetch(s0);
  for (long long s = s0; s < s1; ++s) {
    __syncthreads();                            // the previous strip's operands are consumed
    stage();
    __syncthreads();
    if (s + 1 < s1) fetch(s + 1);               // in flight during this strip's MFMAs
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int px = 16 * wv + 4 * ks + lk;     // this lane's k (pixel of the strip)
      float av[NO];
#pragma unroll
      for (int a = 0; a < NO; ++a) av[a] = gs[(16 * a + li) * DW_GS + px];          // A[i = o][k]
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int ky = tap / 3, kx = tap - 3 * ky;
        float bv[NC];
#pragma unroll
        for (int b = 0; b < NC; ++b) bv[b] = xs[((16 * b + li) * 3 + ky) * DW_XS + px + kx];   // B[k][j = c]
#pragma unroll
        for (int a = 0; a < NO; ++a)
#pragma unroll
          for (int b = 0; b < NC; ++b) acc[a][tap][b] = mfma16(av[a], bv[b], acc[a][tap][b]);
      }
    }
  }
  // D[i = o (row)][j = c (column)]: lane holds o = 16 a + 4 lk + r, c = 16 b + li
  float* red = lds;
  __syncthreads();
  for (int w = 0; w < DK_THREADS / 64; ++w) {
    if (wv == w) {
#pragma unroll
      for (int a = 0; a < NO; ++a)
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
#pragma unroll
          for (int b = 0; b < NC; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int o = 16 * a + 4 * lk + r, c = 16 * b + li;
              float* p = red + (o * CI + c) * 9 + tap;
              *p = (w == 0 ? 0.f : *p) + acc[a][tap][b][r];
            }
    }
    __syncthreads();
  }
  for (int k = threadIdx.x; k < CO * CI * 9; k += DK_THREADS) partial[(size_t)blockIdx.x * CO * CI * 9 + k] = red[k];
}

static int dk_blocks() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 256;
  return cus * 8;
}

}  // namespace vfd

using namespace vfd;

extern "C" {

int vfd_dec_conv_supported(int N, int CI, int CO, int H, int W) {
  const bool ch = (CI == 16 || CI == 32) && (CO == 16 || CO == 32);
  return N > 0 && ch && H > 0 && W > 0 && W % 64 == 0 && (long long)N * (CI > CO ? CI : CO) * (H + 2) * (W + 2) < (1LL << 31);
}

int vfd_dec_conv_wgrad_blocks(int N, int H, int W) { (void)N; (void)H; (void)W; return dk_blocks() / 4; }

#define DK_DISPATCH(KERNEL, ...)                                                            \
  do {                                                                                      \
    if (CI == 16 && CO == 16) KERNEL<16, 16><<<grid, DK_THREADS, 0, s>>>(__VA_ARGS__);      \
    else if (CI == 16 && CO == 32) KERNEL<16, 32><<<grid, DK_THREADS, 0, s>>>(__VA_ARGS__); \
    else if (CI == 32 && CO == 16) KERNEL<32, 16><<<grid, DK_THREADS, 0, s>>>(__VA_ARGS__); \
    else KERNEL<32, 32><<<grid, DK_THREADS, 0, s>>>(__VA_ARGS__);                           \
  } while (0)

int vfd_dec_conv_fwd(const float* xp, const float* w, const float* bias, float* y, int N, int CI, int CO, int H, int W,
                     void* stream) {
  VFD_REQUIRE(vfd_dec_conv_supported(N, CI, CO, H, W), "dec_conv: unsupported shape (CI, CO in {16, 32}, W %% 64 == 0)");
  VFD_REQUIRE(xp && w && bias && y && ((uintptr_t)y & 15) == 0, "dec_conv_fwd: bad argument");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_DEC_CONV, s);
  const long long ntile = (long long)N * H * (W / 16);
  const long long need = (ntile + 3) / 4;
  const unsigned grid = (unsigned)(need < dk_blocks() ? need : dk_blocks());
  DK_DISPATCH(dconv_fwd_k, xp, w, bias, y, N, H, W);
  return fail_launch("dec_conv_fwd");
}

int vfd_dec_conv_bwd(const float* dy, const float* xp, const float* w, float* dxp, float* partial, int N, int CI, int CO,
                     int H, int W, void* stream) {
  VFD_REQUIRE(vfd_dec_conv_supported(N, CI, CO, H, W), "dec_conv: unsupported shape (CI, CO in {16, 32}, W %% 64 == 0)");
  VFD_REQUIRE(dy && w && (!partial || xp), "dec_conv_bwd: bad argument");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_DEC_CONV, s);
  if (dxp) {
    const long long ntile = (long long)N * (H + 2) * ((W + 2 + 15) / 16);
    const long long need = (ntile + 3) / 4;
    const unsigned grid = (unsigned)(need < dk_blocks() ? need : dk_blocks());
    DK_DISPATCH(dconv_dgrad_k, dy, w, dxp, N, H, W);
  }
  if (partial) {
    VFD_REQUIRE(W % DW_S == 0, "dec_conv_bwd: weight gradient needs W %% %d == 0", DW_S);
    const unsigned grid = (unsigned)vfd_dec_conv_wgrad_blocks(N, H, W);
    const long long nstrip = (long long)N * H * (W / DW_S);
    const long long per = (nstrip + grid - 1) / grid;
    DK_DISPATCH(dconv_wgrad_k, dy, xp, partial, N, H, W, per);
  }
  return fail_launch("dec_conv_bwd");
}

}  // extern "C"
