// K4 — fused view synthesis for gfx950 (reference: models/geometry/geometry_util.py:33-82,
// models/geometry/view_rendering.py:30-82, 118-198).
//
// Per target camera the reference runs 8 independent warps (2 temporal, 3 frames x 2 spatial
// neighbours), each a backproject -> matmul -> divide -> grid_sample(bilinear) + grid_sample
// (nearest) -> NaN fix -> OOB mask -> (intensity alignment: two masked global reductions) chain,
// ~15 ATen launches and ~20 full-resolution intermediates per warp.  Here every pixel
// back-projects its depth once and evaluates all warps in registers:
//   view_stats_k    per-warp moments for intensity alignment (fp64 block partials)
//   view_finalize_k means / stds / batch-wide "empty overlap" skip per warp
//   view_apply_k    normalised warps, temporal planes, overlap sums -> the 20 output planes
//   view_bwd_k      d depth (all warps summed per pixel, no atomics) and d (K T)[:3] partials
// Source images (3 frames x N cameras) stay L2/MALL resident; nothing but inputs and the
// output planes touches HBM.
#include "vfd_common.h"

namespace vfd {

constexpr int VPPT = 1;          // pixels per thread in the reduction kernels
constexpr int VBLK = 256;

struct WarpEntry {
  int fslot, src, oslot;         // frame slot, source camera (-1: unused), overlap slot (-1: temporal)
};

// Index conventions: bt = blockIdx.y = b * cam_count + target slot (per-target arrays);
// br = b * N + cam (whole-rig arrays: colours, masks).
struct Target {
  int bt, b, cam;
  size_t br;
};
__device__ __forceinline__ Target target_of(const vfd_view_desc& d, int by) {
  Target t;
  t.bt = by;
  t.b = t.bt / d.cam_count;
  t.cam = d.cam_begin + t.bt % d.cam_count;
  t.br = (size_t)t.b * d.N + t.cam;
  return t;
}

__device__ __forceinline__ WarpEntry warp_entry(const vfd_view_desc& d, int cam, int w) {
  const int* t = d.warp_tab + (cam * d.n_warp + w) * 3;
  return {t[0], t[1], t[2]};
}

// Back-projected point of pixel p (geometry_util.py:56-64).
__device__ __forceinline__ void backproject(const float* __restrict__ iK, float depth, int x, int y,
                                            float* X, float* ray) {
  float fx = (float)x, fy = (float)y;
  ray[0] = iK[0] * fx + iK[1] * fy + iK[2];
  ray[1] = iK[4] * fx + iK[5] * fy + iK[6];
  ray[2] = iK[8] * fx + iK[9] * fy + iK[10];
  X[0] = depth * ray[0];
  X[1] = depth * ray[1];
  X[2] = depth * ray[2];
}

struct WarpSample {
  float a, b, den;       // uvw numerators and w + 1e-7
  float ix, iy;
  float img[3];
  float cm;              // (~OOB) * nearest(mask)
  Bilinear bl;
};

// A warp sample in three steps, so a kernel can put the gathers of several warps in flight before
// it uses any of them (the gathers hit L2 / MALL; issued one by one behind branches they ran as
// serial round trips):
//   warp_geo    reproject (geometry_util.py:66-81) + grid_sample coordinates; no memory access
//   warp_fetch  the 12 bilinear taps + the nearest mask value as unconditional loads (out-of-range
//               and non-finite taps read element 0 and are dropped by warp_combine)
//   warp_combine get_virtual_image (view_rendering.py:61-82): taps in fixed order, NaN -> 2.0, OOB mask
struct WarpGeo {
  float a, b, den, ix, iy;
  Bilinear bl;
  int ni;                // nearest tap, -1 when out of range / non-finite
  bool oob;
};

struct WarpTex {
  float v[3][4];         // channel x tap (nw, ne, sw, se)
  float m;               // nearest mask value
};

__device__ __forceinline__ WarpGeo warp_geo(const float* __restrict__ Mw, const float* X, int H, int W) {
  WarpGeo g;
  g.a = Mw[0] * X[0] + Mw[1] * X[1] + Mw[2] * X[2] + Mw[3];
  g.b = Mw[4] * X[0] + Mw[5] * X[1] + Mw[6] * X[2] + Mw[7];
  const float c = Mw[8] * X[0] + Mw[9] * X[1] + Mw[10] * X[2] + Mw[11];
  g.den = c + 1e-7f;
  const float u = g.a / g.den, v = g.b / g.den;
  const float gx = (u / (float)(W - 1) - 0.5f) * 2.f;
  const float gy = (v / (float)(H - 1) - 0.5f) * 2.f;
  g.ix = unnorm_ac(gx, W);
  g.iy = unnorm_ac(gy, H);
  g.bl = bilinear_taps(g.ix, g.iy, W, H);
  g.ni = nearest_index(g.ix, g.iy, W, H);
  g.oob = (gx > 1.f) || (gx < -1.f) || (gy > 1.f) || (gy < -1.f);
  return g;
}

__device__ __forceinline__ void warp_fetch(const WarpGeo& g, const float* __restrict__ img,
                                           const float* __restrict__ msk, int W, int HW, WarpTex& t) {
  const int base = g.bl.y0 * W + g.bl.x0;
  const int off[4] = {0, 1, W, W + 1};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = g.bl.in[k] ? base + off[k] : 0;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) t.v[ch][k] = img[ch * HW + i];
  }
  t.m = msk[g.ni >= 0 ? g.ni : 0];
}

__device__ __forceinline__ WarpSample warp_combine(const WarpGeo& g, const WarpTex& t) {
  WarpSample s;
  s.a = g.a;
  s.b = g.b;
  s.den = g.den;
  s.ix = g.ix;
  s.iy = g.iy;
  s.bl = g.bl;
  if (!g.bl.finite) {
    s.img[0] = s.img[1] = s.img[2] = 2.f;   // NaN -> 2.0 (view_rendering.py:73-75)
    s.cm = 0.f;
    return s;
  }
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) acc += g.bl.in[k] ? t.v[ch][k] * g.bl.w[k] : 0.f;
    s.img[ch] = acc;
  }
  const float mv = g.ni >= 0 ? t.m : 0.f;
  s.cm = (g.oob ? 0.f : 1.f) * mv;
  return s;
}

__device__ __forceinline__ WarpSample warp_sample(const float* __restrict__ Mw, const float* X,
                                                  const float* __restrict__ img, const float* __restrict__ msk,
                                                  int H, int W) {
  const WarpGeo g = warp_geo(Mw, X, H, W);
  WarpTex t;
  warp_fetch(g, img, msk, W, H * W, t);
  return warp_combine(g, t);
}

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* lds) {
  // 256-thread block, returns the total in thread 0
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) lds[w] = v;
  __syncthreads();
  T t = 0;
  if (threadIdx.x == 0) t = lds[0] + lds[1] + lds[2] + lds[3];
  return t;
}

// Reduce N values (N a power of two <= 64) over the 64 lanes of a wave without LDS or barriers:
// full butterflies for offsets >= N, then value-halving butterflies (each lane keeps half of its
// values); lane L ends with the wave total of v[L % N].
template <int N>
__device__ __forceinline__ float wave_reduce_n(float (&v)[N]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 32; o >= N; o >>= 1)
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += __shfl_xor(v[i], o, 64);
#pragma unroll
  for (int o = N / 2; o >= 1; o >>= 1) {
    const bool up = (lane & o) != 0;
#pragma unroll
    for (int i = 0; i < o; ++i) {
      const float a = v[i], b = v[i + o];
      v[i] = (up ? b : a) + __shfl_xor(up ? a : b, o, 64);
    }
  }
  return v[0];
}

// ------------------------------------------------------------------------------ stats
// partial layout [B*N][n_warp*8 + 2][nblk * 4 waves] floats (per-wave sums; column-major so each
// reduction reads one contiguous column):
//   per warp (8 slots): count(3 per masked pixel), sum w*m, sum r*m, sum w, sum w^2, 0, 0, 0;
//   per camera: sum r, sum r^2.  No barriers: every wave writes its own row.
__global__ __launch_bounds__(VBLK) void view_stats_k(vfd_view_desc d, const float* __restrict__ depth,
                                                     const float* __restrict__ invK, const float* __restrict__ M,
                                                     const float* __restrict__ mask, float* __restrict__ partial) {
  const uint3 bi = xcd_tile();         // XCD-contiguous pixel blocks: a band of rows per XCD's L2
  const Target tg = target_of(d, (int)bi.y);
  const int bn = tg.bt, b = tg.b, cam = tg.cam;
  const int HW = d.H * d.W;
  const int nrow = gridDim.x * (VBLK / 64);
  const int stride = d.n_warp * 8 + 2;
  const int lane = threadIdx.x & 63;
  // column-major partials: column c of camera slot bn is partial[(bn * stride + c) * nrow + row]
  const int row = bi.x * (VBLK / 64) + (threadIdx.x >> 6);
  float* out = partial + (size_t)bn * stride * nrow + row;
  const float* ref = d.color[0] + tg.br * 3 * HW;
  const float* rmask = mask + tg.br * HW;
  float X[VPPT][3], rv[VPPT][3], rm[VPPT];
  int pix[VPPT];
#pragma unroll
  for (int k = 0; k < VPPT; ++k) {
    pix[k] = bi.x * VBLK * VPPT + k * VBLK + threadIdx.x;
    float ray[3];
    const bool in = pix[k] < HW;
    const int pk = in ? pix[k] : 0;
    backproject(invK + bn * 16, depth[(size_t)bn * HW + pk], pk % d.W, pk / d.W, X[k], ray);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) rv[k][ch] = in ? ref[ch * HW + pk] : 0.f;
    rm[k] = rmask[pk];
  }
  {
    float v[2] = {0.f, 0.f};
#pragma unroll
    for (int k = 0; k < VPPT; ++k)
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        v[0] += rv[k][ch];
        v[1] += rv[k][ch] * rv[k][ch];
      }
    const float s = wave_reduce_n<2>(v);
    if (lane < 2) out[(size_t)(d.n_warp * 8 + lane) * nrow] = s;
  }
  const bool live = pix[0] < HW;
  for (int w0 = 0; w0 < d.n_warp; w0 += 2) {
    // the gathers of two warps in flight together; a missing / unused warp reads camera 0
    WarpEntry e[2];
    WarpGeo g[2];
    WarpTex t[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int w = w0 + j < d.n_warp ? w0 + j : w0;
      e[j] = warp_entry(d, cam, w);
      const int src = e[j].src >= 0 ? e[j].src : 0, fs = e[j].src >= 0 ? e[j].fslot : 0;
      const size_t sbn = (size_t)b * d.N + src;
      g[j] = warp_geo(M + ((size_t)bn * d.n_warp + w) * 12, X[0], d.H, d.W);
      warp_fetch(g[j], d.color[fs] + sbn * 3 * HW, mask + sbn * HW, d.W, HW, t[j]);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int w = w0 + j;
      if (w >= d.n_warp) break;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (e[j].src >= 0 && live) {
        const WarpSample s = warp_combine(g[j], t[j]);
        const float mf = (rm[0] * s.cm) != 0.f ? 1.f : 0.f;
        acc[0] += 3.f * mf;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
          const float wv = s.img[ch];
          acc[1] += wv * mf;
          acc[2] += rv[0][ch] * mf;
          acc[3] += wv;
          acc[4] += wv * wv;
        }
      }
      const float sm = wave_reduce_n<8>(acc);
      if (lane < 8) out[(size_t)(w * 8 + lane) * nrow] = sm;
    }
  }
}

// coef [B,N,n_warp,4] = (w_mean, w_std, s_mean, s_std); w_std = -1 marks a skipped warp
// (any sample of the batch without overlap -> warp returned unnormalised, view_rendering.py:50-53)
__global__ __launch_bounds__(512) void view_finalize_k(vfd_view_desc d, const float* __restrict__ partial, int nblk,
                                                       float* __restrict__ coef) {
  // one block per (target slot, warp); wave j < 7 reduces column j (contiguous, fp64) in parallel
  __shared__ double sl[8];
  const int cam = blockIdx.x / d.n_warp, w = blockIdx.x % d.n_warp;
  const int stride = d.n_warp * 8 + 2;
  const double n_all = 3.0 * d.H * d.W;
  const int lane = threadIdx.x & 63, j = threadIdx.x >> 6;
  bool skip = false;
  for (int b = 0; b < d.B; ++b) {
    const size_t bn = (size_t)b * d.cam_count + cam;
    if (j < 7) {
      const int col = j < 5 ? w * 8 + j : d.n_warp * 8 + (j - 5);
      const float* pc = partial + (bn * stride + col) * nblk;
      double acc = 0.0;
      for (int k = lane; k < nblk; k += 64) acc += (double)pc[k];
      acc = wave_sum(acc);
      if (lane == 0) sl[j] = acc;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double s[7];
      for (int i = 0; i < 7; ++i) s[i] = sl[i];
      if (s[0] == 0.0) skip = true;
      const double mw = s[1] / (s[0] + 1e-8);
      const double ms = s[2] / (s[0] + 1e-8);
      double vw = (s[4] - 2.0 * mw * s[3] + n_all * mw * mw) / n_all;
      double vs = (s[6] - 2.0 * ms * s[5] + n_all * ms * ms) / n_all;
      vw = vw < 0.0 ? 0.0 : vw;
      vs = vs < 0.0 ? 0.0 : vs;
      float* c = coef + (bn * d.n_warp + w) * 4;
      c[0] = (float)mw;
      c[1] = sqrtf((float)vw + 1e-16f);
      c[2] = (float)ms;
      c[3] = sqrtf((float)vs + 1e-16f);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && (skip || !d.intensity_align)) {
    for (int b = 0; b < d.B; ++b) coef[(((size_t)b * d.cam_count + cam) * d.n_warp + w) * 4 + 1] = -1.f;
  }
}

// ------------------------------------------------------------------------------ apply
__global__ __launch_bounds__(VBLK) void view_apply_k(vfd_view_desc d, const float* __restrict__ depth,
                                                     const float* __restrict__ invK, const float* __restrict__ M,
                                                     const float* __restrict__ mask, const float* __restrict__ coef,
                                                     float* __restrict__ color, float* __restrict__ cmask,
                                                     float* __restrict__ ovl, float* __restrict__ omask) {
  const uint3 bi = xcd_tile();
  const Target tg = target_of(d, (int)bi.y);
  const int bn = tg.bt, b = tg.b, cam = tg.cam;
  const int HW = d.H * d.W;
  const int p = bi.x * VBLK + threadIdx.x;
  if (p >= HW) return;
  float X[3], ray[3];
  backproject(invK + bn * 16, depth[(size_t)bn * HW + p], p % d.W, p / d.W, X, ray);
  const int T = d.n_temporal, F = d.n_overlap;
  // temporal warps: their own planes
  for (int w = 0; w < d.n_warp; ++w) {
    const WarpEntry e = warp_entry(d, cam, w);
    if (e.src < 0 || e.oslot >= 0) continue;
    const size_t sbn = (size_t)b * d.N + e.src;
    const float* cf = coef + ((size_t)bn * d.n_warp + w) * 4;
    WarpSample s = warp_sample(M + ((size_t)bn * d.n_warp + w) * 12, X, d.color[e.fslot] + sbn * 3 * HW,
                               mask + sbn * HW, d.H, d.W);
    float* co = color + (((size_t)bn * T + w) * 3) * HW;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      float o = s.img[ch];
      if (cf[1] >= 0.f) o = ((o - cf[0]) / (cf[1] + 1e-8f) * cf[3] + cf[2]) * s.cm;
      co[ch * HW + p] = o;
    }
    cmask[((size_t)bn * T + w) * HW + p] = s.cm;
  }
  // overlap slots: sum over the spatial neighbours in table order
  for (int slot = 0; slot < F; ++slot) {
    float acc[3] = {0.f, 0.f, 0.f}, macc = 0.f;
    for (int w = 0; w < d.n_warp; ++w) {
      const WarpEntry e = warp_entry(d, cam, w);
      if (e.src < 0 || e.oslot != slot) continue;
      const size_t sbn = (size_t)b * d.N + e.src;
      const float* cf = coef + ((size_t)bn * d.n_warp + w) * 4;
      WarpSample s = warp_sample(M + ((size_t)bn * d.n_warp + w) * 12, X, d.color[e.fslot] + sbn * 3 * HW,
                                 mask + sbn * HW, d.H, d.W);
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        float o = s.img[ch];
        if (cf[1] >= 0.f) o = ((o - cf[0]) / (cf[1] + 1e-8f) * cf[3] + cf[2]) * s.cm;
        acc[ch] = acc[ch] + o;
      }
      macc = macc + s.cm;
    }
    float* oo = ovl + (((size_t)bn * F + slot) * 3) * HW;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) oo[ch * HW + p] = acc[ch];
    omask[((size_t)bn * F + slot) * HW + p] = macc;
  }
}

// ------------------------------------------------------------------------------ backward
// partial layout [B*N][n_warp][16][nblk * 4 waves] floats (d (K T)[:3] per warp in slots 0..11,
// column-major for contiguous reductions).
__global__ __launch_bounds__(VBLK) void view_bwd_k(vfd_view_desc d, const float* __restrict__ depth,
                                                   const float* __restrict__ invK, const float* __restrict__ M,
                                                   const float* __restrict__ mask, const float* __restrict__ coef,
                                                   const float* __restrict__ g_color, const float* __restrict__ g_ovl,
                                                   float* __restrict__ d_depth, float* __restrict__ partial) {
  const uint3 bi = xcd_tile();
  const Target tg = target_of(d, (int)bi.y);
  const int bn = tg.bt, b = tg.b, cam = tg.cam;
  const int HW = d.H * d.W;
  const int nrow = gridDim.x * (VBLK / 64);
  const int row = bi.x * (VBLK / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int T = d.n_temporal, F = d.n_overlap;
  float X[VPPT][3], ray[VPPT][3], dd[VPPT];
  int pix[VPPT];
#pragma unroll
  for (int k = 0; k < VPPT; ++k) {
    pix[k] = bi.x * VBLK * VPPT + k * VBLK + threadIdx.x;
    dd[k] = 0.f;
    const int pk = pix[k] < HW ? pix[k] : 0;
    backproject(invK + bn * 16, depth[(size_t)bn * HW + pk], pk % d.W, pk / d.W, X[k], ray[k]);
  }
  const bool live = pix[0] < HW;
  const int pk = live ? pix[0] : 0;
  constexpr int VB = 1;     // warps per batch (2 measured slower: 99 VGPRs cost occupancy)
  for (int w0 = 0; w0 < d.n_warp; w0 += VB) {
    // a warp's gathers (taps, mask, incoming gradient) in flight together
    const float* gsrc[VB];
    WarpGeo g[VB];
    WarpTex t[VB];
    float gv[VB][3];
#pragma unroll
    for (int j = 0; j < VB; ++j) {
      const int w = w0 + j < d.n_warp ? w0 + j : w0;
      const WarpEntry e = warp_entry(d, cam, w);
      gsrc[j] = nullptr;
      if (e.src >= 0)
        gsrc[j] = e.oslot < 0 ? (g_color ? g_color + (((size_t)bn * T + w) * 3) * HW : nullptr)
                              : (g_ovl ? g_ovl + (((size_t)bn * F + e.oslot) * 3) * HW : nullptr);
      if (w0 + j >= d.n_warp) gsrc[j] = nullptr;
      const int src = e.src >= 0 ? e.src : 0, fs = e.src >= 0 ? e.fslot : 0;
      const size_t sbn = (size_t)b * d.N + src;
      g[j] = warp_geo(M + ((size_t)bn * d.n_warp + w) * 12, X[0], d.H, d.W);
      warp_fetch(g[j], d.color[fs] + sbn * 3 * HW, mask + sbn * HW, d.W, HW, t[j]);
      const float* gp = gsrc[j] ? gsrc[j] : depth;   // any readable plane when unused
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) gv[j][ch] = gp[(gsrc[j] ? ch * HW : 0) + pk];
    }
#pragma unroll
    for (int j = 0; j < VB; ++j) {
      const int w = w0 + j;
      if (w >= d.n_warp) break;
      float dM[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) dM[i] = 0.f;
      if (gsrc[j] && live && g[j].bl.finite) {
        const float* Mw = M + ((size_t)bn * d.n_warp + w) * 12;
        const float* cf = coef + ((size_t)bn * d.n_warp + w) * 4;
        const bool norm = cf[1] >= 0.f;
        const WarpSample s = warp_combine(g[j], t[j]);
        const float x0 = floorf(s.ix), y0 = floorf(s.iy);
        const float x1 = x0 + 1.f, y1 = y0 + 1.f;
        float gix = 0.f, giy = 0.f;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
          float gg = gv[j][ch];
          if (norm) gg = gg * s.cm * cf[3] / (cf[1] + 1e-8f);
          const float* v = t[j].v[ch];
          if (s.bl.in[0]) { gix -= v[0] * (y1 - s.iy) * gg; giy -= v[0] * (x1 - s.ix) * gg; }
          if (s.bl.in[1]) { gix += v[1] * (y1 - s.iy) * gg; giy -= v[1] * (s.ix - x0) * gg; }
          if (s.bl.in[2]) { gix -= v[2] * (s.iy - y0) * gg; giy += v[2] * (x1 - s.ix) * gg; }
          if (s.bl.in[3]) { gix += v[3] * (s.iy - y0) * gg; giy += v[3] * (s.ix - x0) * gg; }
        }
        // grid_sampler unnormalise -> (u/(W-1) - 0.5)*2 -> a/den
        const float dgx = gix * ((float)(d.W - 1) / 2.f);
        const float dgy = giy * ((float)(d.H - 1) / 2.f);
        const float du = dgx * 2.f / (float)(d.W - 1);
        const float dv = dgy * 2.f / (float)(d.H - 1);
        const float da = du / s.den, db = dv / s.den;
        const float dden = -(du * s.a + dv * s.b) / (s.den * s.den);
        const float Xh[4] = {X[0][0], X[0][1], X[0][2], 1.f};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          dM[q] += da * Xh[q];
          dM[4 + q] += db * Xh[q];
          dM[8 + q] += dden * Xh[q];
        }
        const float dX0 = da * Mw[0] + db * Mw[4] + dden * Mw[8];
        const float dX1 = da * Mw[1] + db * Mw[5] + dden * Mw[9];
        const float dX2 = da * Mw[2] + db * Mw[6] + dden * Mw[10];
        dd[0] += dX0 * ray[0][0] + dX1 * ray[0][1] + dX2 * ray[0][2];
      }
      const float sm = wave_reduce_n<16>(dM);
      if (lane < 12) partial[(((size_t)bn * d.n_warp + w) * 16 + lane) * nrow + row] = sm;
    }
  }
#pragma unroll
  for (int k = 0; k < VPPT; ++k)
    if (pix[k] < HW) d_depth[(size_t)bn * HW + pix[k]] = dd[k];
}

__global__ __launch_bounds__(256) void view_bwd_reduce_k(const float* __restrict__ partial, int nblk, int n_warp,
                                                         float* __restrict__ dM) {
  // one block per output (bn, w, j): fp64 block reduction over the per-block partials
  __shared__ double lds[4];
  const int i = blockIdx.x;
  const int j = i % 12, w = (i / 12) % n_warp, bn = i / (12 * n_warp);
  double s = 0.0;
  for (int k = threadIdx.x; k < nblk; k += blockDim.x) s += (double)partial[(((size_t)bn * n_warp + w) * 16 + j) * nblk + k];
  s = block_sum_all(s, lds);
  if (threadIdx.x == 0) dM[i] = (float)s;
}

}  // namespace vfd

// ================================================================================== C ABI
using namespace vfd;

static int check_view(const vfd_view_desc* d) {
  VFD_REQUIRE(d != nullptr, "null descriptor");
  VFD_REQUIRE(d->B > 0 && d->N > 0 && d->H > 1 && d->W > 1, "bad view sizes");
  VFD_REQUIRE(d->n_warp > 0 && d->n_warp <= 16, "n_warp=%d unsupported", d->n_warp);
  VFD_REQUIRE(d->n_temporal >= 0 && d->n_temporal <= 3 && d->n_overlap >= 0 && d->n_overlap <= 4, "bad frame counts");
  VFD_REQUIRE(d->warp_tab != nullptr && d->color[0] != nullptr, "warp table / colour not set");
  VFD_REQUIRE(d->cam_count > 0 && d->cam_begin >= 0 && d->cam_begin + d->cam_count <= d->N, "bad target range");
  return VFD_OK;
}

static unsigned view_red_blocks(const vfd_view_desc* d) { return cdiv((size_t)d->H * d->W, VBLK * VPPT); }

extern "C" {

size_t vfd_view_workspace_bytes(const vfd_view_desc* d) {
  const size_t nrow = (size_t)view_red_blocks(d) * (VBLK / 64);
  const size_t stats = (size_t)d->B * d->cam_count * nrow * (d->n_warp * 8 + 2) * sizeof(float);
  const size_t bwd = (size_t)d->B * d->cam_count * nrow * d->n_warp * 16 * sizeof(float);
  return stats > bwd ? stats : bwd;
}

int vfd_view_fwd(const vfd_view_desc* d, const float* depth, const float* invK, const float* M, const float* mask,
                 float* color, float* cmask, float* ovl, float* omask, float* coef, void* ws, size_t ws_bytes,
                 void* stream) {
  int st = check_view(d);
  if (st) return st;
  VFD_REQUIRE(ws_bytes >= vfd_view_workspace_bytes(d), "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const unsigned nblk = view_red_blocks(d);
  {
    ProfScope ps(K_VIEW_STATS, s);          // the op: per-wave partials + their reduction
    view_stats_k<<<dim3(nblk, d->B * d->cam_count), VBLK, 0, s>>>(*d, depth, invK, M, mask, (float*)ws);
    if ((st = fail_launch("view_stats"))) return st;
    view_finalize_k<<<d->cam_count * d->n_warp, 512, 0, s>>>(*d, (const float*)ws, nblk * (VBLK / 64), coef);
  }
  if ((st = fail_launch("view_finalize"))) return st;
  {
    ProfScope ps(K_VIEW_APPLY, s);
    view_apply_k<<<dim3(cdiv((size_t)d->H * d->W, VBLK), d->B * d->cam_count), VBLK, 0, s>>>(*d, depth, invK, M, mask, coef,
                                                                                     color, cmask, ovl, omask);
  }
  return fail_launch("view_apply");
}

int vfd_view_bwd(const vfd_view_desc* d, const float* depth, const float* invK, const float* M, const float* mask,
                 const float* coef, const float* g_color, const float* g_ovl, float* d_depth, float* d_M, void* ws,
                 size_t ws_bytes, void* stream) {
  int st = check_view(d);
  if (st) return st;
  VFD_REQUIRE(ws_bytes >= vfd_view_workspace_bytes(d), "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const unsigned nblk = view_red_blocks(d);
  {
    ProfScope ps(K_VIEW_BWD, s);            // the op: per-wave partials + their reduction
    view_bwd_k<<<dim3(nblk, d->B * d->cam_count), VBLK, 0, s>>>(*d, depth, invK, M, mask, coef, g_color, g_ovl, d_depth,
                                                        (float*)ws);
    if ((st = fail_launch("view_bwd"))) return st;
    const int n = d->B * d->cam_count * d->n_warp * 12;
    view_bwd_reduce_k<<<n, 256, 0, s>>>((const float*)ws, nblk * (VBLK / 64), d->n_warp, d_M);
  }
  return fail_launch("view_bwd_reduce");
}

}  // extern "C"
