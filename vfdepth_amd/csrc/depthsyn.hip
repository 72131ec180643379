// Depth synthesis at an augmented view (reference: models/geometry/view_rendering.py:84-116,
// 201-241; selected by training.aug_depth, models/vfdepth.py:48-49).
//
// For every target camera c and source slot s (sources rel_cam_list[c] + [c]), the reference
// back-projects the source depth map, takes the z of those points in the augmented view of c
// (T = E_aug[c]^-1 E[src]), and backward-warps that map into the augmented view through the
// augmented view's own predicted depth (bilinear, zeros padding, align_corners), with a nearest
// mask lookup, NaN -> 2.0, OOB masking and a [min, max] clamp whose replaced values carry no
// gradient.  Here one thread per target pixel evaluates all S sources: the source "z map" is never
// materialised (each bilinear tap recomputes its source pixel's z from the source depth).
//   depth_syn_fwd_k  -> tform_depth [B,N,S,H,W], tform_mask [B,N,S,H,W]
//   depth_syn_bwd_k  -> d aug_depth (per pixel, summed over the sources: no atomics) and
//                       d depth of the sources (the bilinear transpose: f32 atomics, or — the
//                       ordered form — exact 128-bit fixed-point integer sums, whose value does
//                       not depend on the order the atomics land in)
#include "vfd_common.h"

namespace vfd {

struct DsSample {
  float a, b, den, ix, iy;
  float z[4];               // source z-map values at the 4 taps (0 when out of range)
  float dz[4];              // d z / d source depth at the taps
  int q[4];                 // tap pixel (or -1)
  Bilinear bl;
  float depth;              // warped depth after the NaN rule and the clamps
  float mask;
  bool pass;                // gradient reaches the sample (finite, not replaced by a bound)
};

// backproject (geometry_util.py:56-64): ray = invK[:3,:3] (x, y, 1); point = depth * ray
__device__ __forceinline__ void ds_ray(const float* __restrict__ iK, int x, int y, float* r) {
  const float fx = (float)x, fy = (float)y;
  r[0] = iK[0] * fx + iK[1] * fy + iK[2];
  r[1] = iK[4] * fx + iK[5] * fy + iK[6];
  r[2] = iK[8] * fx + iK[9] * fy + iK[10];
}

__device__ __forceinline__ DsSample ds_sample(const vfd_depthsyn_desc& d, const float* __restrict__ M,
                                              const float* __restrict__ zr, const float* X,
                                              const float* __restrict__ sdepth, const float* __restrict__ smask,
                                              const float* __restrict__ siK) {
  DsSample s;
  const int H = d.H, W = d.W;
  // reproject with (K_src @ T^-1)[:3] (geometry_util.py:66-81)
  s.a = M[0] * X[0] + M[1] * X[1] + M[2] * X[2] + M[3];
  s.b = M[4] * X[0] + M[5] * X[1] + M[6] * X[2] + M[7];
  const float c = M[8] * X[0] + M[9] * X[1] + M[10] * X[2] + M[11];
  s.den = c + 1e-7f;
  const float u = s.a / s.den, v = s.b / s.den;
  const float gx = (u / (float)(W - 1) - 0.5f) * 2.f;
  const float gy = (v / (float)(H - 1) - 0.5f) * 2.f;
  s.ix = unnorm_ac(gx, W);
  s.iy = unnorm_ac(gy, H);
  s.bl = bilinear_taps(s.ix, s.iy, W, H);
  if (!s.bl.finite) {                          // NaN -> 2.0 depth, mask 0 (view_rendering.py:103-106)
    s.depth = 2.f;
    s.mask = 0.f;
    s.pass = false;
  } else {
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      s.q[k] = -1;
      s.z[k] = s.dz[k] = 0.f;
      if (!s.bl.in[k]) continue;
      const int x = s.bl.x0 + (k & 1), y = s.bl.y0 + (k >> 1);
      const int q = y * W + x;
      float r[3];
      ds_ray(siK, x, y, r);
      const float dq = sdepth[q];
      // z row of T @ [depth * ray; 1] (view_rendering.py:91-93)
      s.z[k] = zr[0] * (dq * r[0]) + zr[1] * (dq * r[1]) + zr[2] * (dq * r[2]) + zr[3];
      s.dz[k] = zr[0] * r[0] + zr[1] * r[1] + zr[2] * r[2];
      s.q[k] = q;
      acc += s.z[k] * s.bl.w[k];
    }
    const int ni = nearest_index(s.ix, s.iy, W, H);
    const float mv = ni >= 0 ? smask[ni] : 0.f;
    const bool oob = (gx > 1.f) || (gx < -1.f) || (gy > 1.f) || (gy < -1.f);
    s.depth = acc;
    s.mask = (oob ? 0.f : 1.f) * mv;
    s.pass = true;
  }
  // range handling (view_rendering.py:111-115): replaced values get the bound and no gradient
  const bool vmin = s.depth > d.min_depth;
  if (!vmin) s.depth = d.min_depth;
  const bool vmax = s.depth < d.max_depth;
  if (!vmax) s.depth = d.max_depth;
  s.mask = s.mask * (vmin ? 1.f : 0.f) * (vmax ? 1.f : 0.f);
  s.pass = s.pass && vmin && vmax;
  return s;
}

__global__ __launch_bounds__(256) void depth_syn_fwd_k(vfd_depthsyn_desc d, const float* __restrict__ aug_depth,
                                                       const float* __restrict__ depth, const float* __restrict__ mask,
                                                       const float* __restrict__ invK, const float* __restrict__ M,
                                                       const float* __restrict__ zrow, float* __restrict__ out_depth,
                                                       float* __restrict__ out_mask) {
  const int HW = d.H * d.W;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int bc = blockIdx.y, b = bc / d.N, c = bc % d.N;
  if (p >= HW) return;
  float r[3], X[3];
  ds_ray(invK + bc * 16, p % d.W, p / d.W, r);
  const float ad = aug_depth[(size_t)bc * HW + p];
  X[0] = ad * r[0];
  X[1] = ad * r[1];
  X[2] = ad * r[2];
  for (int s = 0; s < d.S; ++s) {
    const size_t o = ((size_t)bc * d.S + s) * HW + p;
    const int src = d.src_tab[c * d.S + s];
    if (src < 0) {
      out_depth[o] = 0.f;
      out_mask[o] = 0.f;
      continue;
    }
    const size_t sb = (size_t)b * d.N + src;
    const DsSample sm = ds_sample(d, M + ((size_t)bc * d.S + s) * 12, zrow + ((size_t)bc * d.S + s) * 4, X,
                                  depth + sb * HW, mask + sb * HW, invK + sb * 16);
    out_depth[o] = sm.depth;
    out_mask[o] = sm.mask;
  }
}

// Ordered (deterministic) accumulation: a contribution v is the signed 128-bit integer
// round-toward-zero(v * 2^DS_FRAC) (exact for |v| >= 2^-DS_FRAC+23, |v| < 2^26), added to the
// pixel's (hi, lo) pair by two 64-bit integer atomics with the low word's carry passed on.
// Integer addition is associative, so the pair ends the same whatever order the adds land in.
// The pair holds sums of magnitude < 2^27 (63 - 36 integer bits in hi); contributions of
// magnitude >= DS_FIXED_MAX (and non-finite ones) take the float atomic instead (ds_fixed_ok), so
// the shift below never leaves [-24, 102] and the integer part cannot overflow from one add.
constexpr int DS_FRAC = 100;
constexpr float DS_FIXED_MAX = 0x1p25f;

__device__ __forceinline__ bool ds_fixed_ok(float v) { return fabsf(v) < DS_FIXED_MAX; }   // false for NaN / inf

__device__ __forceinline__ void ds_fixed_add(unsigned long long* __restrict__ cell, float v) {
  const unsigned u = __float_as_uint(v);
  const int ex = (int)((u >> 23) & 255u);
  if (ex == 0) return;                               // zero / denormal (< 1.2e-38): nothing
  const int sh = ex - 127 - 23 + DS_FRAC;            // v = m * 2^(ex - 150), m < 2^24
  if (sh <= -24) return;                             // below the fixed-point resolution
  const unsigned long long m = (unsigned long long)((u & 0x7FFFFFu) | 0x800000u);
  unsigned long long lo, hi;
  if (sh < 0) {
    lo = m >> -sh;
    hi = 0ull;
  } else if (sh < 64) {
    lo = m << sh;
    hi = sh > 40 ? m >> (64 - sh) : 0ull;
  } else {
    lo = 0ull;
    hi = m << (sh - 64);                               // sh <= 102 for |v| < 2^26
  }
  if (u >> 31) {                                     // two's complement of the 128-bit value
    lo = ~lo + 1ull;
    hi = ~hi + (lo == 0ull ? 1ull : 0ull);
  }
  const unsigned long long old = atomicAdd(cell + 1, lo);
  const unsigned long long carry = old + lo < old ? 1ull : 0ull;
  atomicAdd(cell, hi + carry);
}

// d_depth from the fixed-point pairs [hi, lo]
__global__ __launch_bounds__(256) void depth_syn_fixed_k(const unsigned long long* __restrict__ acc, size_t n,
                                                         float* __restrict__ d_depth) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long hi = (long long)acc[2 * i];
  const unsigned long long lo = acc[2 * i + 1];
  // + the non-finite / out-of-range contributions, which went to d_depth itself (0 when there were none)
  d_depth[i] = (float)((double)hi * 0x1p-36 + (double)lo * 0x1p-100) + d_depth[i];
}

template <bool ORDERED>
__global__ __launch_bounds__(256) void depth_syn_bwd_k(vfd_depthsyn_desc d, const float* __restrict__ aug_depth,
                                                       const float* __restrict__ depth, const float* __restrict__ mask,
                                                       const float* __restrict__ invK, const float* __restrict__ M,
                                                       const float* __restrict__ zrow, const float* __restrict__ g,
                                                       float* __restrict__ d_aug, float* __restrict__ d_depth,
                                                       unsigned long long* __restrict__ fixed) {
  const int HW = d.H * d.W;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int bc = blockIdx.y, b = bc / d.N, c = bc % d.N;
  if (p >= HW) return;
  float r[3], X[3];
  ds_ray(invK + bc * 16, p % d.W, p / d.W, r);
  const float ad = aug_depth[(size_t)bc * HW + p];
  X[0] = ad * r[0];
  X[1] = ad * r[1];
  X[2] = ad * r[2];
  float dad = 0.f;
  for (int s = 0; s < d.S; ++s) {
    const int src = d.src_tab[c * d.S + s];
    if (src < 0) continue;
    const float gv = g[((size_t)bc * d.S + s) * HW + p];
    const size_t sb = (size_t)b * d.N + src;
    const float* Mw = M + ((size_t)bc * d.S + s) * 12;
    const DsSample sm = ds_sample(d, Mw, zrow + ((size_t)bc * d.S + s) * 4, X, depth + sb * HW, mask + sb * HW,
                                  invK + sb * 16);
    if (!sm.pass || gv == 0.f) continue;
    // values: d z_k = g w_k -> d source depth = g w_k dz/ddepth (grid_sampler_2d_backward's scatter)
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (sm.q[k] >= 0) {
        const float v = gv * sm.bl.w[k] * sm.dz[k];
        if (ORDERED && ds_fixed_ok(v)) ds_fixed_add(fixed + 2 * (sb * HW + sm.q[k]), v);
        else atomicAdd(d_depth + sb * HW + sm.q[k], v);   // (ordered form: non-finite or |v| >= 2^25 only)
      }
    // coordinates (zeros padding: out-of-range taps contribute nothing)
    const float x0 = floorf(sm.ix), y0 = floorf(sm.iy), x1 = x0 + 1.f, y1 = y0 + 1.f;
    float gix = 0.f, giy = 0.f;
    if (sm.bl.in[0]) { gix -= sm.z[0] * (y1 - sm.iy) * gv; giy -= sm.z[0] * (x1 - sm.ix) * gv; }
    if (sm.bl.in[1]) { gix += sm.z[1] * (y1 - sm.iy) * gv; giy -= sm.z[1] * (sm.ix - x0) * gv; }
    if (sm.bl.in[2]) { gix -= sm.z[2] * (sm.iy - y0) * gv; giy += sm.z[2] * (x1 - sm.ix) * gv; }
    if (sm.bl.in[3]) { gix += sm.z[3] * (sm.iy - y0) * gv; giy += sm.z[3] * (sm.ix - x0) * gv; }
    const float du = gix * ((float)(d.W - 1) / 2.f) * 2.f / (float)(d.W - 1);
    const float dv = giy * ((float)(d.H - 1) / 2.f) * 2.f / (float)(d.H - 1);
    const float da = du / sm.den, db = dv / sm.den;
    const float dden = -(du * sm.a + dv * sm.b) / (sm.den * sm.den);
    const float dX0 = da * Mw[0] + db * Mw[4] + dden * Mw[8];
    const float dX1 = da * Mw[1] + db * Mw[5] + dden * Mw[9];
    const float dX2 = da * Mw[2] + db * Mw[6] + dden * Mw[10];
    dad += dX0 * r[0] + dX1 * r[1] + dX2 * r[2];
  }
  d_aug[(size_t)bc * HW + p] = dad;
}

static int check_ds(const vfd_depthsyn_desc* d) {
  VFD_REQUIRE(d && d->B > 0 && d->N > 0 && d->H > 1 && d->W > 1 && d->S > 0 && d->src_tab,
              "depth_syn: bad descriptor");
  return VFD_OK;
}

}  // namespace vfd

using namespace vfd;

extern "C" {

int vfd_depth_syn_fwd(const vfd_depthsyn_desc* d, const float* aug_depth, const float* depth, const float* mask,
                      const float* invK, const float* M, const float* zrow, float* out_depth, float* out_mask,
                      void* stream) {
  if (int e = check_ds(d)) return e;
  VFD_REQUIRE(aug_depth && depth && mask && invK && M && zrow && out_depth && out_mask, "depth_syn_fwd: null argument");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_DEPTH_SYN_FWD, s);
  dim3 grid(cdiv(d->H * d->W, 256), d->B * d->N);
  depth_syn_fwd_k<<<grid, 256, 0, s>>>(*d, aug_depth, depth, mask, invK, M, zrow, out_depth, out_mask);
  return fail_launch("depth_syn_fwd");
}

int vfd_depth_syn_bwd(const vfd_depthsyn_desc* d, const float* aug_depth, const float* depth, const float* mask,
                      const float* invK, const float* M, const float* zrow, const float* g, float* d_aug,
                      float* d_depth, void* stream) {
  if (int e = check_ds(d)) return e;
  VFD_REQUIRE(aug_depth && depth && mask && invK && M && zrow && g && d_aug && d_depth, "depth_syn_bwd: null argument");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_DEPTH_SYN_BWD, s);
  zero_async(d_depth, sizeof(float) * (size_t)d->B * d->N * d->H * d->W, s);
  dim3 grid(cdiv(d->H * d->W, 256), d->B * d->N);
  depth_syn_bwd_k<false><<<grid, 256, 0, s>>>(*d, aug_depth, depth, mask, invK, M, zrow, g, d_aug, d_depth, nullptr);
  return fail_launch("depth_syn_bwd");
}

size_t vfd_depth_syn_bwd_ordered_workspace(const vfd_depthsyn_desc* d) {
  if (!d || d->B <= 0 || d->N <= 0 || d->H <= 0 || d->W <= 0) return 0;
  return (size_t)d->B * d->N * d->H * d->W * 2 * sizeof(unsigned long long);
}

int vfd_depth_syn_bwd_ordered(const vfd_depthsyn_desc* d, const float* aug_depth, const float* depth,
                              const float* mask, const float* invK, const float* M, const float* zrow,
                              const float* g, float* d_aug, float* d_depth, void* workspace, size_t ws_bytes,
                              void* stream) {
  if (int e = check_ds(d)) return e;
  VFD_REQUIRE(aug_depth && depth && mask && invK && M && zrow && g && d_aug && d_depth && workspace,
              "depth_syn_bwd_ordered: null argument");
  const size_t need = vfd_depth_syn_bwd_ordered_workspace(d);
  VFD_REQUIRE(ws_bytes >= need, "depth_syn_bwd_ordered: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_DEPTH_SYN_BWD, s);
  auto* fixed = (unsigned long long*)workspace;
  zero_async(fixed, need, s);
  zero_async(d_depth, sizeof(float) * (size_t)d->B * d->N * d->H * d->W, s);
  dim3 grid(cdiv(d->H * d->W, 256), d->B * d->N);
  depth_syn_bwd_k<true><<<grid, 256, 0, s>>>(*d, aug_depth, depth, mask, invK, M, zrow, g, d_aug, d_depth, fixed);
  const size_t n = (size_t)d->B * d->N * d->H * d->W;
  depth_syn_fixed_k<<<(unsigned)cdiv((long long)n, 256), 256, 0, s>>>(fixed, n, d_depth);
  return fail_launch("depth_syn_bwd_ordered");
}

}  // extern "C"
