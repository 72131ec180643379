// Multi-level feature aggregation at the fusion level (reference: network/fusion_depthnet.py:53-63,
// fusion_posenet.py:55-66):  agg = LReLU_0.1( conv1x1( cat(f_l, up(f_l+1), ..., up(f_4)) ) ).
// The 1x1 conv is linear and bilinear upsampling (align_corners=True) acts per channel, so
// conv1x1(cat(f_l, up(f_k)...)) = W_l f_l + sum_k up(W_k f_k) + b.  The caller applies each W_k at
// its own (lower) resolution; this kernel upsamples the 256-channel products, adds them with the
// bias and applies the LeakyReLU in one pass (ATen's bilinear upsample kernel parallelises over
// output pixels only and took ~0.5-0.9 ms per level at config 2).
#include "vfd_common.h"

namespace vfd {

struct UpLevel {
  const float* src;
  int h, w;
};

__device__ __forceinline__ float up_ac(const float* __restrict__ plane, int hs, int ws, int h, int w, int y, int x) {
  // F.interpolate(..., [h, w], mode='bilinear', align_corners=True) at (y, x) (ATen UpSample.h)
  int y0, y1, x0, x1;
  float ly, lx;
  if (hs == h) { y0 = y1 = y; ly = 0.f; } else {
    const float sy = h > 1 ? (float)(hs - 1) / (float)(h - 1) : 0.f;
    const float fy = sy * (float)y;
    y0 = min((int)floorf(fy), hs - 1);
    ly = fminf(fmaxf(fy - (float)y0, 0.f), 1.f);
    y1 = y0 + (y0 < hs - 1 ? 1 : 0);
  }
  if (ws == w) { x0 = x1 = x; lx = 0.f; } else {
    const float sx = w > 1 ? (float)(ws - 1) / (float)(w - 1) : 0.f;
    const float fx = sx * (float)x;
    x0 = min((int)floorf(fx), ws - 1);
    lx = fminf(fmaxf(fx - (float)x0, 0.f), 1.f);
    x1 = x0 + (x0 < ws - 1 ? 1 : 0);
  }
  const float top = (1.f - lx) * plane[y0 * ws + x0] + lx * plane[y0 * ws + x1];
  const float bot = (1.f - lx) * plane[y1 * ws + x0] + lx * plane[y1 * ws + x1];
  return (1.f - ly) * top + ly * bot;
}

template <int NL>
__global__ __launch_bounds__(256) void aggregate_fwd_k(int BN, int C, int h, int w, const float* __restrict__ base,
                                                       UpLevel l0, UpLevel l1, UpLevel l2,
                                                       const float* __restrict__ bias, float* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t n = (size_t)BN * C * h * w;
  if (i >= n) return;
  const int x = i % w, y = (i / w) % h;
  const size_t plane = i / ((size_t)h * w);          // n * C + c
  const int c = plane % C;
  float v = base[i];
  const UpLevel lv[3] = {l0, l1, l2};
#pragma unroll
  for (int k = 0; k < NL; ++k) v += up_ac(lv[k].src + plane * lv[k].h * lv[k].w, lv[k].h, lv[k].w, h, w, y, x);
  v += bias[c];
  out[i] = v > 0.f ? v : v * 0.1f;
}

}  // namespace vfd

using namespace vfd;

namespace vfd {

// source index / weight of output row y under align_corners=True resizing from n_src to n (the
// forward's arithmetic: up_ac)
__device__ __forceinline__ void up_axis(int n_src, int n, int y, int* y0, int* y1, float* l) {
  if (n_src == n) { *y0 = *y1 = y; *l = 0.f; return; }
  const float sy = n > 1 ? (float)(n_src - 1) / (float)(n - 1) : 0.f;
  const float fy = sy * (float)y;
  *y0 = min((int)floorf(fy), n_src - 1);
  *l = fminf(fmaxf(fy - (float)*y0, 0.f), 1.f);
  *y1 = *y0 + (*y0 < n_src - 1 ? 1 : 0);
}

// Backward of the align_corners bilinear upsample as a separable gather (the forward weight of
// source (ys, xs) for output (y, x) is wy(y, ys) * wx(x, xs)): pass 1 sums each output row over
// the columns whose taps name xs, pass 2 sums those over the rows whose taps name ys; every sum
// in a fixed order (ATen's backward scatters with atomics).  Candidate indices come from the
// scale, then the forward's exact taps decide.
__device__ __forceinline__ void up_range(int s, int n_src, int n, int* lo, int* hi) {
  if (n_src == n) { *lo = *hi = s; return; }
  const float sc = n > 1 ? (float)(n_src - 1) / (float)(n - 1) : 0.f;
  if (!(sc > 0.f)) { *lo = 0; *hi = n - 1; return; }
  *lo = max(0, (int)floorf((float)(s - 1) / sc) - 1);
  *hi = min(n - 1, (int)ceilf((float)(s + 1) / sc) + 1);
}

__device__ __forceinline__ float up_weight(int n_src, int n, int y, int s) {
  int y0, y1;
  float l;
  up_axis(n_src, n, y, &y0, &y1, &l);
  return (y0 == s ? 1.f - l : 0.f) + (y1 == s ? l : 0.f);
}

// tmp[p][y][xs] = sum_x wx(x, xs) g[p][y][x]
__global__ __launch_bounds__(256) void up_ac_bwd_x_k(const float* __restrict__ g, float* __restrict__ tmp,
                                                     long long planes, int h, int w, int ws) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;       // (y, xs) of the plane
  if (j >= h * ws) return;
  const int y = j / ws, xs = j - y * ws;
  int lo, hi;
  up_range(xs, ws, w, &lo, &hi);
  for (long long p = blockIdx.y; p < planes; p += gridDim.y) {
    const float* gr = g + (p * h + y) * w;
    float acc = 0.f;
    // unconditional loads (a zero weight adds nothing): a load behind the weight test waited for
    // each candidate in turn
#pragma unroll 4
    for (int x = lo; x <= hi; ++x) acc += up_weight(ws, w, x, xs) * gr[x];
    tmp[p * h * ws + j] = acc;
  }
}

// dsrc[p][ys][xs] = sum_y wy(y, ys) tmp[p][y][xs]
__global__ __launch_bounds__(256) void up_ac_bwd_y_k(const float* __restrict__ tmp, float* __restrict__ dsrc,
                                                     long long planes, int h, int hs, int ws) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;       // (ys, xs) of the plane
  if (j >= hs * ws) return;
  const int ys = j / ws, xs = j - ys * ws;
  int lo, hi;
  up_range(ys, hs, h, &lo, &hi);
  for (long long p = blockIdx.y; p < planes; p += gridDim.y) {
    const float* tp = tmp + p * h * ws + xs;
    float acc = 0.f;
#pragma unroll 4
    for (int y = lo; y <= hi; ++y) acc += up_weight(hs, h, y, ys) * tp[(size_t)y * ws];
    dsrc[p * hs * ws + j] = acc;
  }
}

// ---- one workgroup per (n, c) plane, for planes whose working set fits LDS (every config here)
// Forward: the plane's level maps are staged in LDS once, so the 4 taps per level of every output
// read LDS instead of L2 (the flat kernel above issued 12 global loads per output element).
// Backward: d = g * LReLU'(out) is written once and kept in LDS; its plane sum (the bias gradient's
// partial) and, per level, the separable gather (rows -> LDS tmp -> columns) all run from LDS.
// Same arithmetic and summation order as aggregate_fwd_k / up_ac_bwd_{x,y}_k.
constexpr int AGG_T = 256;
constexpr int AGG_BT = 512;                        // backward: more lanes per plane for its serial phases
constexpr int AGG_LDS_MAX = 64 * 1024;

struct AggLevels {
  const float* src[3];
  float* dst[3];
  int hs[3], ws[3];
};

template <int NL>
__global__ __launch_bounds__(AGG_T) void aggregate_plane_fwd_k(int C, int h, int w, const float* __restrict__ base,
                                                               AggLevels lv, const float* __restrict__ bias,
                                                               float* __restrict__ out) {
  extern __shared__ float agg_sm[];
  const size_t p = blockIdx.x;                       // n * C + c
  float* lp[3] = {agg_sm, agg_sm, agg_sm};
  int off = 0;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int n = lv.hs[k] * lv.ws[k];
    lp[k] = agg_sm + off;
    const float* src = lv.src[k] + p * n;
    for (int i = threadIdx.x; i < n; i += AGG_T) lp[k][i] = src[i];
    off += n;
  }
  __syncthreads();
  const float bc = bias[p % C];
  const int hw = h * w;
  const float* bp = base + p * hw;
  float* op = out + p * hw;
  constexpr int U = 4;                               // base loads in flight per thread
  for (int i0 = threadIdx.x; i0 < hw; i0 += U * AGG_T) {
    float bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) bv[u] = bp[min(i0 + u * AGG_T, hw - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * AGG_T;
      if (i < hw) {
        const int x = i % w, y = i / w;
        float v = bv[u];
#pragma unroll
        for (int k = 0; k < NL; ++k) v += up_ac(lp[k], lv.hs[k], lv.ws[k], h, w, y, x);
        v += bc;
        op[i] = v > 0.f ? v : v * 0.1f;
      }
    }
  }
}

// floats of the backward's gather scratch: h x the widest level
__device__ __forceinline__ int agg_tmp_floats(int h, const AggLevels& lv, int nl) {
  int m = 0;
  for (int k = 0; k < nl; ++k) m = max(m, lv.ws[k]);
  return h * m;
}

template <int NL>
__global__ __launch_bounds__(AGG_BT) void aggregate_plane_bwd_k(int h, int w, const float* __restrict__ g,
                                                               const float* __restrict__ out, float* __restrict__ d,
                                                               AggLevels lv, float* __restrict__ psum) {
  extern __shared__ float agg_sm[];
  __shared__ float wsum[AGG_BT / 64];
  const size_t p = blockIdx.x;
  const int hw = h * w;
  float* dp = agg_sm;
  float* tmp = agg_sm + hw;
  float s = 0.f;
  constexpr int U = 4;                               // loads in flight per thread
  const float* gp = g + p * hw;
  const float* opl = out + p * hw;
  for (int i0 = threadIdx.x; i0 < hw; i0 += U * AGG_BT) {
    float gv[U], ov[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(i0 + u * AGG_BT, hw - 1);
      gv[u] = gp[i];
      ov[u] = opl[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * AGG_BT;
      if (i < hw) {
        const float dv = gv[u] * (ov[u] > 0.f ? 1.f : 0.1f);
        d[p * hw + i] = dv;
        dp[i] = dv;
        s += dv;
      }
    }
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < AGG_BT / 64; ++k) t += wsum[k];
    psum[p] = t;
  }
  // per level: the forward's taps of every output column / row and each source's candidate
  // range, once per plane in LDS (the gathers then read tables instead of redoing up_axis per tap)
  int* xt0 = reinterpret_cast<int*>(tmp + agg_tmp_floats(h, lv, NL));
  int* xt1 = xt0 + w;
  float* xl = reinterpret_cast<float*>(xt1 + w);
  int* yt0 = reinterpret_cast<int*>(xl + w);
  int* yt1 = yt0 + h;
  float* yl = reinterpret_cast<float*>(yt1 + h);
  int* xlo = reinterpret_cast<int*>(yl + h);
  int* xhi = xlo + w;
  int* ylo = xhi + w;
  int* yhi = ylo + h;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int hs = lv.hs[k], ws = lv.ws[k];
    for (int i = threadIdx.x; i < w + h; i += AGG_BT) {
      if (i < w) {
        up_axis(ws, w, i, &xt0[i], &xt1[i], &xl[i]);
        if (i < ws) up_range(i, ws, w, &xlo[i], &xhi[i]);
      } else {
        const int y = i - w;
        up_axis(hs, h, y, &yt0[y], &yt1[y], &yl[y]);
        if (y < hs) up_range(y, hs, h, &ylo[y], &yhi[y]);
      }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < h * ws; j += AGG_BT) {
      const int y = j / ws, xs = j - y * ws;
      const int lo = xlo[xs], hi = xhi[xs];
      const float* gr = dp + y * w;
      float acc = 0.f;
      for (int x = lo; x <= hi; ++x) {
        const float l = xl[x];
        acc += ((xt0[x] == xs ? 1.f - l : 0.f) + (xt1[x] == xs ? l : 0.f)) * gr[x];
      }
      tmp[j] = acc;
    }
    __syncthreads();
    float* dst = lv.dst[k] + p * hs * ws;
    for (int j = threadIdx.x; j < hs * ws; j += AGG_BT) {
      const int ys = j / ws, xs = j - ys * ws;
      const int lo = ylo[ys], hi = yhi[ys];
      float acc = 0.f;
      for (int y = lo; y <= hi; ++y) {
        const float l = yl[y];
        acc += ((yt0[y] == ys ? 1.f - l : 0.f) + (yt1[y] == ys ? l : 0.f)) * tmp[y * ws + xs];
      }
      dst[j] = acc;
    }
    __syncthreads();
  }
}

// ---- channels-last inputs (config 3: the bf16 1x1-conv products of the channels-last encoders),
// NCHW fp32 output as aggregate_plane_fwd_k.  A workgroup takes (image n, row y, 32 columns, 64
// channels): lanes run over channels for the base / level reads (128-B bf16 rows), the results go
// through an LDS tile [64][33] and leave with lanes over columns (128-B NCHW rows).  Per element the
// arithmetic of aggregate_fwd_k / up_ac (level taps of the same fp32 values in the same order):
// bit-identical to the NCHW path on the fp32-converted inputs.
constexpr int AGC_X = 32, AGC_C = 64;
#ifndef VFD_AGC_U
#define VFD_AGC_U 2                                // columns per thread in flight (of 8)
#endif
#ifndef VFD_AGC_PAIR
#define VFD_AGC_PAIR 1                             // channel pairs per lane (aggregate_cl2_fwd_k)
#endif

struct AggLevelsT {
  const void* src[3];
  int hs[3], ws[3];
};

template <int NL, typename TI>
__global__ __launch_bounds__(256) void aggregate_cl_fwd_k(int C, int h, int w, const TI* __restrict__ base,
                                                          AggLevelsT lv, const float* __restrict__ bias,
                                                          float* __restrict__ out) {
  __shared__ float tile[AGC_C][AGC_X + 1];
  const int ncx = (w + AGC_X - 1) / AGC_X;
  const int x0 = (blockIdx.x % ncx) * AGC_X, c0 = (blockIdx.x / ncx) * AGC_C;
  const int y = blockIdx.y;
  const long long n = blockIdx.z;
  const int cl = threadIdx.x & (AGC_C - 1), xq = threadIdx.x >> 6;
  const int c = c0 + cl;
  if (c < C) {
    // the vertical taps of every level (the same for all of this thread's columns)
    int ya[3], yb[3];
    float lyv[3];
#pragma unroll
    for (int k = 0; k < NL; ++k) up_axis(lv.hs[k], h, y, &ya[k], &yb[k], &lyv[k]);
    const TI* bp = base + ((n * h + y) * w) * C + c;
    const float bc = bias[c];
#pragma unroll VFD_AGC_U
    for (int xl = xq; xl < AGC_X; xl += 4) {
      const int x = x0 + xl;
      if (x >= w) break;
      float v = ld1(bp + (size_t)x * C);
#pragma unroll
      for (int k = 0; k < NL; ++k) {
        const int hs = lv.hs[k], ws = lv.ws[k];
        int xa, xb;
        float lx;
        up_axis(ws, w, x, &xa, &xb, &lx);
        const TI* lp = reinterpret_cast<const TI*>(lv.src[k]) + (n * hs * ws) * C + c;
        const float top = (1.f - lx) * ld1(lp + ((size_t)ya[k] * ws + xa) * C) + lx * ld1(lp + ((size_t)ya[k] * ws + xb) * C);
        const float bot = (1.f - lx) * ld1(lp + ((size_t)yb[k] * ws + xa) * C) + lx * ld1(lp + ((size_t)yb[k] * ws + xb) * C);
        v += (1.f - lyv[k]) * top + lyv[k] * bot;
      }
      v += bc;
      tile[cl][xl] = v > 0.f ? v : v * 0.1f;
    }
  }
  __syncthreads();
  const int xo = threadIdx.x & (AGC_X - 1), cr = threadIdx.x >> 5;
  if (x0 + xo < w) {
#pragma unroll
    for (int j = 0; j < AGC_C / 8; ++j) {
      const int cc = cr + 8 * j;
      if (c0 + cc < C) out[((n * C + c0 + cc) * h + y) * w + x0 + xo] = tile[cc][xo];
    }
  }
}

// The same with a channel pair per lane (C even, 8-B / 4-B aligned maps): 128 channels per
// workgroup, one 8-B fp32 / 4-B bf16 load per tap and pair — half the load instructions; each
// channel's arithmetic is aggregate_cl_fwd_k's.
__device__ __forceinline__ float2 agc_ld2(const float* p) { return *reinterpret_cast<const float2*>(p); }
__device__ __forceinline__ float2 agc_ld2(const __bf16* p) {
  const uint32_t u = *reinterpret_cast<const uint32_t*>(p);
  return make_float2(__uint_as_float(u << 16), __uint_as_float(u & 0xFFFF0000u));
}

constexpr int AGC2_C = 2 * AGC_C;

template <int NL, typename TI>
__global__ __launch_bounds__(256) void aggregate_cl2_fwd_k(int C, int h, int w, const TI* __restrict__ base,
                                                           AggLevelsT lv, const float* __restrict__ bias,
                                                           float* __restrict__ out) {
  __shared__ float tile[AGC2_C][AGC_X + 1];
  const int ncx = (w + AGC_X - 1) / AGC_X;
  const int x0 = (blockIdx.x % ncx) * AGC_X, c0 = (blockIdx.x / ncx) * AGC2_C;
  const int y = blockIdx.y;
  const long long n = blockIdx.z;
  const int cl = threadIdx.x & (AGC_C - 1), xq = threadIdx.x >> 6;
  const int c = c0 + 2 * cl;
  if (c < C) {
    int ya[3], yb[3];
    float lyv[3];
#pragma unroll
    for (int k = 0; k < NL; ++k) up_axis(lv.hs[k], h, y, &ya[k], &yb[k], &lyv[k]);
    const TI* bp = base + ((n * h + y) * w) * C + c;
    const float bc0 = bias[c], bc1 = bias[c + 1];
#pragma unroll VFD_AGC_U
    for (int xl = xq; xl < AGC_X; xl += 4) {
      const int x = x0 + xl;
      if (x >= w) break;
      const float2 b = agc_ld2(bp + (size_t)x * C);
      float v0 = b.x, v1 = b.y;
#pragma unroll
      for (int k = 0; k < NL; ++k) {
        const int hs = lv.hs[k], ws = lv.ws[k];
        int xa, xb;
        float lx;
        up_axis(ws, w, x, &xa, &xb, &lx);
        const TI* lp = reinterpret_cast<const TI*>(lv.src[k]) + (n * hs * ws) * C + c;
        const float2 p00 = agc_ld2(lp + ((size_t)ya[k] * ws + xa) * C), p01 = agc_ld2(lp + ((size_t)ya[k] * ws + xb) * C);
        const float2 p10 = agc_ld2(lp + ((size_t)yb[k] * ws + xa) * C), p11 = agc_ld2(lp + ((size_t)yb[k] * ws + xb) * C);
        const float top0 = (1.f - lx) * p00.x + lx * p01.x, bot0 = (1.f - lx) * p10.x + lx * p11.x;
        const float top1 = (1.f - lx) * p00.y + lx * p01.y, bot1 = (1.f - lx) * p10.y + lx * p11.y;
        v0 += (1.f - lyv[k]) * top0 + lyv[k] * bot0;
        v1 += (1.f - lyv[k]) * top1 + lyv[k] * bot1;
      }
      v0 += bc0;
      v1 += bc1;
      tile[2 * cl][xl] = v0 > 0.f ? v0 : v0 * 0.1f;
      tile[2 * cl + 1][xl] = v1 > 0.f ? v1 : v1 * 0.1f;
    }
  }
  __syncthreads();
  const int xo = threadIdx.x & (AGC_X - 1), cr = threadIdx.x >> 5;
  if (x0 + xo < w) {
#pragma unroll 4
    for (int j = 0; j < AGC2_C / 8; ++j) {
      const int cc = cr + 8 * j;
      if (c0 + cc < C) out[((n * C + c0 + cc) * h + y) * w + x0 + xo] = tile[cc][xo];
    }
  }
}

}  // namespace vfd

namespace vfd {
// NCHW fp32 [n][C][hw] -> channels-last [n][hw][C] of TO (one rounding): the aggregation's input
// gradients handed back in the layout / dtype of its channels-last inputs (what autograd's cast and
// the convolution backward's layout copy would otherwise do in two passes).  64 x 64 tiles through
// LDS: lanes over pixels on the read, over channels on the write.
template <typename TO>
__global__ __launch_bounds__(256) void nchw_to_nhwc_k(const float* __restrict__ x, TO* __restrict__ y, int C, int hw) {
  __shared__ float t[64][65];
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const long long n = blockIdx.z;
  const int l = threadIdx.x & 63, r = threadIdx.x >> 6;
#pragma unroll 4
  for (int k = r; k < 64; k += 4)
    if (c0 + k < C && p0 + l < hw) t[k][l] = x[(n * C + c0 + k) * hw + p0 + l];
  __syncthreads();
#pragma unroll 4
  for (int k = r; k < 64; k += 4)
    if (p0 + k < hw && c0 + l < C) y[(n * hw + p0 + k) * C + c0 + l] = (TO)t[l][k];
}
}  // namespace vfd

extern "C" int vfd_nchw_to_nhwc(const float* x, void* y, long long n, int C, int hw, int dtype_out, void* stream) {
  VFD_REQUIRE(x && y && n > 0 && n < 65536 && C > 0 && hw > 0 && (dtype_out == 0 || dtype_out == 1),
              "nchw_to_nhwc: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  vfd::ProfScope ps(vfd::K_LAYOUT_COPY, s);
  const dim3 grid((unsigned)((hw + 63) / 64), (unsigned)((C + 63) / 64), (unsigned)n);
  if (dtype_out == 1) vfd::nchw_to_nhwc_k<__bf16><<<grid, 256, 0, s>>>(x, (__bf16*)y, C, hw);
  else vfd::nchw_to_nhwc_k<float><<<grid, 256, 0, s>>>(x, (float*)y, C, hw);
  return vfd::fail_launch("nchw_to_nhwc");
}

// base / levels channels-last [BN, h, w, C] / [BN, hs, ws, C] of dtype (0 fp32, 1 bf16), out NCHW fp32
extern "C" int vfd_aggregate_fwd_cl(int BN, int C, int h, int w, const void* base, int n_levels,
                                    const void* const* levels, const int* level_hw, const float* bias, float* out,
                                    int dtype, void* stream) {
  VFD_REQUIRE(BN > 0 && C > 0 && h > 0 && w > 0 && base && bias && out && (dtype == 0 || dtype == 1) && BN < 65536 &&
                  h < 65536,
              "aggregate_fwd_cl: bad arguments");
  VFD_REQUIRE(n_levels >= 0 && n_levels <= 3, "up to 3 upsampled levels supported (got %d)", n_levels);
  vfd::AggLevelsT lv{};
  for (int k = 0; k < n_levels; ++k) {
    lv.src[k] = levels[k];
    lv.hs[k] = level_hw[2 * k];
    lv.ws[k] = level_hw[2 * k + 1];
    VFD_REQUIRE(lv.src[k] && lv.hs[k] > 0 && lv.ws[k] > 0, "aggregate_fwd_cl: level %d", k);
  }
  hipStream_t s = (hipStream_t)stream;
  vfd::ProfScope ps(vfd::K_AGGREGATE, s);
  // channel pairs when every map allows the 2-element loads
  uintptr_t al = (uintptr_t)base;
  for (int k = 0; k < n_levels; ++k) al |= (uintptr_t)lv.src[k];
  const bool pair = VFD_AGC_PAIR && C % 2 == 0 && (al & (dtype ? 3 : 7)) == 0;
  const int cpb = pair ? vfd::AGC2_C : vfd::AGC_C;
  const dim3 grid((unsigned)(((w + vfd::AGC_X - 1) / vfd::AGC_X) * ((C + cpb - 1) / cpb)), (unsigned)h, (unsigned)BN);
#define VFD_AGC(NL, T)                                                                                           \
  if (pair) vfd::aggregate_cl2_fwd_k<NL, T><<<grid, 256, 0, s>>>(C, h, w, (const T*)base, lv, bias, out);        \
  else vfd::aggregate_cl_fwd_k<NL, T><<<grid, 256, 0, s>>>(C, h, w, (const T*)base, lv, bias, out)
#define VFD_AGC_T(T)                      \
  switch (n_levels) {                     \
    case 0: VFD_AGC(0, T); break;         \
    case 1: VFD_AGC(1, T); break;         \
    case 2: VFD_AGC(2, T); break;         \
    default: VFD_AGC(3, T); break;        \
  }
  if (dtype == 1) {
    VFD_AGC_T(__bf16)
  } else {
    VFD_AGC_T(float)
  }
#undef VFD_AGC_T
#undef VFD_AGC
  return vfd::fail_launch("aggregate_fwd_cl");
}

extern "C" int vfd_aggregate_bwd(int BN, int C, int h, int w, const float* g, const float* out, float* d,
                                 int n_levels, float* const* dlevels, const int* level_hw, float* psum, void* stream) {
  VFD_REQUIRE(BN > 0 && C > 0 && h > 0 && w > 0 && g && out && d && psum, "aggregate_bwd: bad arguments");
  VFD_REQUIRE(n_levels >= 0 && n_levels <= 3, "up to 3 upsampled levels supported (got %d)", n_levels);
  vfd::AggLevels lv{};
  int wsmax = 0;
  for (int k = 0; k < n_levels; ++k) {
    lv.dst[k] = dlevels[k];
    lv.hs[k] = level_hw[2 * k];
    lv.ws[k] = level_hw[2 * k + 1];
    VFD_REQUIRE(lv.dst[k] && lv.hs[k] > 0 && lv.ws[k] > 0 && lv.hs[k] <= h && lv.ws[k] <= w, "aggregate_bwd: level %d", k);
    wsmax = lv.ws[k] > wsmax ? lv.ws[k] : wsmax;
  }
  const size_t lds = ((size_t)h * w + (size_t)h * wsmax + 5 * (size_t)(w + h)) * 4;   // d, tmp, tap tables
  VFD_REQUIRE(lds <= (size_t)vfd::AGG_LDS_MAX, "aggregate_bwd: plane %dx%d too large for LDS", h, w);
  hipStream_t s = (hipStream_t)stream;
  vfd::ProfScope ps(vfd::K_UPSAMPLE_BWD, s);
  const unsigned nb = (unsigned)((long long)BN * C);
  switch (n_levels) {
    case 0: vfd::aggregate_plane_bwd_k<0><<<nb, vfd::AGG_BT, lds, s>>>(h, w, g, out, d, lv, psum); break;
    case 1: vfd::aggregate_plane_bwd_k<1><<<nb, vfd::AGG_BT, lds, s>>>(h, w, g, out, d, lv, psum); break;
    case 2: vfd::aggregate_plane_bwd_k<2><<<nb, vfd::AGG_BT, lds, s>>>(h, w, g, out, d, lv, psum); break;
    default: vfd::aggregate_plane_bwd_k<3><<<nb, vfd::AGG_BT, lds, s>>>(h, w, g, out, d, lv, psum); break;
  }
  return vfd::fail_launch("aggregate_bwd");
}

extern "C" int vfd_upsample_ac_bwd(const float* g, float* dsrc, float* tmp, long long planes, int h, int w, int hs,
                                   int ws, void* stream) {
  VFD_REQUIRE(g && dsrc && tmp && planes > 0 && h > 0 && w > 0 && hs > 0 && ws > 0 && hs <= h && ws <= w,
              "upsample_ac_bwd: bad sizes");
  hipStream_t s = (hipStream_t)stream;
  vfd::ProfScope ps(vfd::K_UPSAMPLE_BWD, s);
  VFD_REQUIRE((long long)h * w < (1LL << 31), "upsample_ac_bwd: plane too large");
  const unsigned gy = (unsigned)(planes < 65535 ? planes : 65535);
  vfd::up_ac_bwd_x_k<<<dim3((unsigned)((h * ws + 255) / 256), gy), 256, 0, s>>>(g, tmp, planes, h, w, ws);
  vfd::up_ac_bwd_y_k<<<dim3((unsigned)((hs * ws + 255) / 256), gy), 256, 0, s>>>(tmp, dsrc, planes, h, hs, ws);
  return vfd::fail_launch("upsample_ac_bwd");
}

extern "C" int vfd_aggregate_fwd(int BN, int C, int h, int w, const float* base, int n_levels,
                                 const float* const* levels, const int* level_hw, const float* bias, float* out,
                                 void* stream) {
  VFD_REQUIRE(BN > 0 && C > 0 && h > 0 && w > 0, "bad aggregate sizes");
  VFD_REQUIRE(n_levels >= 0 && n_levels <= 3, "up to 3 upsampled levels supported (got %d)", n_levels);
  UpLevel lv[3] = {{nullptr, 1, 1}, {nullptr, 1, 1}, {nullptr, 1, 1}};
  for (int k = 0; k < n_levels; ++k) lv[k] = {levels[k], level_hw[2 * k], level_hw[2 * k + 1]};
  hipStream_t s = (hipStream_t)stream;
  const size_t n = (size_t)BN * C * h * w;
  ProfScope ps(K_AGGREGATE, s);
  size_t lds = 0;
  AggLevels al{};
  for (int k = 0; k < n_levels; ++k) {
    al.src[k] = lv[k].src;
    al.hs[k] = lv[k].h;
    al.ws[k] = lv[k].w;
    lds += (size_t)lv[k].h * lv[k].w * 4;
  }
  if (lds <= (size_t)AGG_LDS_MAX / 2) {          // per-plane form (levels staged in LDS)
    const unsigned nb = (unsigned)((long long)BN * C);
    switch (n_levels) {
      case 0: aggregate_plane_fwd_k<0><<<nb, AGG_T, lds, s>>>(C, h, w, base, al, bias, out); break;
      case 1: aggregate_plane_fwd_k<1><<<nb, AGG_T, lds, s>>>(C, h, w, base, al, bias, out); break;
      case 2: aggregate_plane_fwd_k<2><<<nb, AGG_T, lds, s>>>(C, h, w, base, al, bias, out); break;
      default: aggregate_plane_fwd_k<3><<<nb, AGG_T, lds, s>>>(C, h, w, base, al, bias, out); break;
    }
    return fail_launch("aggregate_fwd");
  }
  switch (n_levels) {
    case 0: aggregate_fwd_k<0><<<cdiv(n, 256), 256, 0, s>>>(BN, C, h, w, base, lv[0], lv[1], lv[2], bias, out); break;
    case 1: aggregate_fwd_k<1><<<cdiv(n, 256), 256, 0, s>>>(BN, C, h, w, base, lv[0], lv[1], lv[2], bias, out); break;
    case 2: aggregate_fwd_k<2><<<cdiv(n, 256), 256, 0, s>>>(BN, C, h, w, base, lv[0], lv[1], lv[2], bias, out); break;
    default: aggregate_fwd_k<3><<<cdiv(n, 256), 256, 0, s>>>(BN, C, h, w, base, lv[0], lv[1], lv[2], bias, out); break;
  }
  return fail_launch("aggregate_fwd");
}
