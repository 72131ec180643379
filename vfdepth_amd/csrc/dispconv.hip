// The depth decoder's disparity head at full resolution: disp = sigmoid(conv3x3_reflect(x) + b)
// with 16 input channels and one output channel (fusion_depthnet.py:117-118, 139-141: the
// ('dispconv', 0) conv2d block, nonlin None, then nn.Sigmoid).  The input arrives already
// reflect-padded (xp [N, 16, H+2, W+2], written by the ELU-pad kernel), so the conv runs with
// padding 0.  MIOpen spends ~170 us forward and ~300 us backward on this one-output-channel conv
// (its solvers are tuned for wide channel counts); each pass here is one sweep over xp:
//
//   disp_conv_fwd_k    thread = 4 consecutive outputs of a row: 16 channels x 3 rows x 6 columns
//                      of xp, 576 FMAs, sigmoid, one 16-B store
//   disp_conv_dgrad_k  thread = 4 consecutive padded positions: d pre = g * s * (1 - s) for the
//                      3 x 6 window of outputs that reach them, 16 channel planes of dxp written
//   disp_conv_wgrad_k  thread = 4 outputs: the 144 weight and 1 bias partial products in
//                      registers, block sums in a fixed order -> partial[block][145] (the caller
//                      sums the blocks: deterministic)
#include "vfd_common.h"

namespace vfd {

constexpr int DC_C = 16;       // input channels
constexpr int DC_E = 4;        // outputs per thread
constexpr int DC_THREADS = 256;

__device__ __forceinline__ float dc_sigmoid(float v) { return 1.f / (1.f + expf(-v)); }

__global__ __launch_bounds__(DC_THREADS) void disp_conv_fwd_k(const float* __restrict__ xp, const float* __restrict__ w,
                                                              const float* __restrict__ bias, float* __restrict__ out,
                                                              int N, int H, int W) {
  const int wq = W / DC_E;
  const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= (long long)N * H * wq) return;
  const int x0 = (int)(j % wq) * DC_E;
  const int y = (int)((j / wq) % H), n = (int)(j / ((long long)wq * H));
  const int wp = W + 2, hp = H + 2;
  float acc[DC_E];
  const float b = bias[0];
#pragma unroll
  for (int e = 0; e < DC_E; ++e) acc[e] = b;
  const float* base = xp + ((size_t)n * DC_C * hp + y) * wp + x0;
#pragma unroll 4
  for (int c = 0; c < DC_C; ++c) {
    const float* pc = base + (size_t)c * hp * wp;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      float r[DC_E + 2];
#pragma unroll
      for (int k = 0; k < DC_E + 2; ++k) r[k] = pc[ky * wp + k];
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const float wv = w[(c * 3 + ky) * 3 + kx];
#pragma unroll
        for (int e = 0; e < DC_E; ++e) acc[e] = fmaf(wv, r[e + kx], acc[e]);
      }
    }
  }
  float4 o;
  o.x = dc_sigmoid(acc[0]);
  o.y = dc_sigmoid(acc[1]);
  o.z = dc_sigmoid(acc[2]);
  o.w = dc_sigmoid(acc[3]);
  *reinterpret_cast<float4*>(out + ((size_t)n * H + y) * W + x0) = o;
}

// d pre-activation at output (n, yy, xx); zero outside the output grid
__device__ __forceinline__ float dc_dpre(const float* __restrict__ g, const float* __restrict__ s, int n, int yy, int xx,
                                         int H, int W) {
  if (yy < 0 || yy >= H || xx < 0 || xx >= W) return 0.f;
  const size_t o = ((size_t)n * H + yy) * W + xx;
  const float sv = s[o];
  return g[o] * (sv * (1.f - sv));
}

__global__ __launch_bounds__(DC_THREADS) void disp_conv_dgrad_k(const float* __restrict__ g, const float* __restrict__ s,
                                                                const float* __restrict__ w, float* __restrict__ dxp,
                                                                int N, int H, int W) {
  const int wp = W + 2, hp = H + 2;
  const int wq = (wp + DC_E - 1) / DC_E;
  const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= (long long)N * hp * wq) return;
  const int X0 = (int)(j % wq) * DC_E;
  const int Y = (int)((j / wq) % hp), n = (int)(j / ((long long)wq * hp));
  // dxp[c][Y][X] = sum_{ky,kx} w[c][ky][kx] * dpre[Y-ky][X-kx]: rows Y-2..Y, columns X0-2..X0+DC_E-1
  float d[3][DC_E + 2];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int k = 0; k < DC_E + 2; ++k) d[r][k] = dc_dpre(g, s, n, Y - 2 + r, X0 - 2 + k, H, W);
  float* base = dxp + ((size_t)n * DC_C * hp + Y) * wp + X0;
  for (int c = 0; c < DC_C; ++c) {
    float acc[DC_E] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const float wv = w[(c * 3 + ky) * 3 + kx];
        // output row Y - ky is d row 2 - ky; output column X - kx is d column (X - X0) + 2 - kx
#pragma unroll
        for (int e = 0; e < DC_E; ++e) acc[e] = fmaf(wv, d[2 - ky][e + 2 - kx], acc[e]);
      }
    float* pc = base + (size_t)c * hp * wp;
#pragma unroll
    for (int e = 0; e < DC_E; ++e)
      if (X0 + e < wp) pc[e] = acc[e];
  }
}

constexpr int DC_NP = DC_C * 9 + 1;     // weight + bias partials

__global__ __launch_bounds__(DC_THREADS) void disp_conv_wgrad_k(const float* __restrict__ g, const float* __restrict__ s,
                                                                const float* __restrict__ xp, float* __restrict__ partial,
                                                                int N, int H, int W) {
  __shared__ float red[DC_THREADS / 64][DC_NP];
  const int wq = W / DC_E;
  const long long j0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = j0 < (long long)N * H * wq;
  const long long j = live ? j0 : 0;
  const int x0 = (int)(j % wq) * DC_E;
  const int y = (int)((j / wq) % H), n = (int)(j / ((long long)wq * H));
  const int wp = W + 2, hp = H + 2;
  float dp[DC_E];
  {
    const size_t o = ((size_t)n * H + y) * W + x0;
    const float4 gv = *reinterpret_cast<const float4*>(g + o);
    const float4 sv = *reinterpret_cast<const float4*>(s + o);
    const float f = live ? 1.f : 0.f;
    dp[0] = f * gv.x * (sv.x * (1.f - sv.x));
    dp[1] = f * gv.y * (sv.y * (1.f - sv.y));
    dp[2] = f * gv.z * (sv.z * (1.f - sv.z));
    dp[3] = f * gv.w * (sv.w * (1.f - sv.w));
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float* base = xp + ((size_t)n * DC_C * hp + y) * wp + x0;
  for (int c = 0; c < DC_C; ++c) {
    const float* pc = base + (size_t)c * hp * wp;
    float acc[9];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      float r[DC_E + 2];
#pragma unroll
      for (int k = 0; k < DC_E + 2; ++k) r[k] = pc[ky * wp + k];
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        float a = 0.f;
#pragma unroll
        for (int e = 0; e < DC_E; ++e) a = fmaf(dp[e], r[e + kx], a);
        acc[ky * 3 + kx] = a;
      }
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const float t = wave_sum(acc[k]);
      if (lane == 0) red[wv][c * 9 + k] = t;
    }
  }
  {
    const float t = wave_sum((dp[0] + dp[1]) + (dp[2] + dp[3]));
    if (lane == 0) red[wv][DC_NP - 1] = t;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < DC_NP; k += blockDim.x)
    partial[(size_t)blockIdx.x * DC_NP + k] = (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]);
}

}  // namespace vfd

using namespace vfd;

extern "C" {

static int dc_check(int N, int C, int H, int W) {
  VFD_REQUIRE(N > 0 && C == DC_C && H > 0 && W > 0 && W % DC_E == 0 && (long long)N * C * (H + 2) * (W + 2) < (1LL << 31),
              "disp_conv: needs %d input channels and W %% %d == 0 (got C=%d, W=%d)", DC_C, DC_E, C, W);
  return VFD_OK;
}

int vfd_disp_conv_supported(int N, int C, int H, int W) {
  return N > 0 && C == DC_C && H > 0 && W > 0 && W % DC_E == 0 && (long long)N * C * (H + 2) * (W + 2) < (1LL << 31);
}

int vfd_disp_conv_wgrad_blocks(int N, int H, int W) {
  return (int)(((long long)N * H * (W / DC_E) + DC_THREADS - 1) / DC_THREADS);
}

int vfd_disp_conv_fwd(const float* xp, const float* w, const float* bias, float* out, int N, int C, int H, int W,
                      void* stream) {
  if (int e = dc_check(N, C, H, W)) return e;
  VFD_REQUIRE(xp && w && bias && out && ((uintptr_t)out & 15) == 0, "disp_conv_fwd: bad argument");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_DISP_CONV, s);
  const long long n = (long long)N * H * (W / DC_E);
  disp_conv_fwd_k<<<(unsigned)((n + DC_THREADS - 1) / DC_THREADS), DC_THREADS, 0, s>>>(xp, w, bias, out, N, H, W);
  return fail_launch("disp_conv_fwd");
}

int vfd_disp_conv_bwd(const float* g, const float* out, const float* xp, const float* w, float* dxp, float* partial,
                      int N, int C, int H, int W, void* stream) {
  if (int e = dc_check(N, C, H, W)) return e;
  VFD_REQUIRE(g && out && w && (((uintptr_t)g | (uintptr_t)out) & 15) == 0 && (!partial || xp),
              "disp_conv_bwd: bad argument");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_DISP_CONV, s);
  if (dxp) {
    const long long n = (long long)N * (H + 2) * ((W + 2 + DC_E - 1) / DC_E);
    disp_conv_dgrad_k<<<(unsigned)((n + DC_THREADS - 1) / DC_THREADS), DC_THREADS, 0, s>>>(g, out, w, dxp, N, H, W);
  }
  if (partial)
    disp_conv_wgrad_k<<<(unsigned)vfd_disp_conv_wgrad_blocks(N, H, W), DC_THREADS, 0, s>>>(g, out, xp, partial, N, H, W);
  return fail_launch("disp_conv_bwd");
}

}  // extern "C"
