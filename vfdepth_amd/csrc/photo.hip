// K5 — photometric losses for gfx950 (reference: models/losses/loss_util.py:6-78,
// single_cam_loss.py:17-65, multi_cam_loss.py:16-59).
//
// The reference evaluates 7 photometric maps per camera (2 reprojection, 2 identity, 1 spatial,
// 2 spatio-temporal), each as ReflectionPad + 5 avg_pool2d + ~20 elementwise ATen kernels, then
// cat/min/argmin/max and three masked means with host syncs.  photo_fwd_k stages the target and
// the 7 predictions of a 16x16 tile (+1 reflect halo) in LDS once and produces every map, the
// argmin selections, the auto-mask, the output planes and the masked-sum partials in one pass.
// photo_bwd_k recomputes the 3x3 moments from a +2 halo and applies the SSIM/L1 chain rule with
// the reflect-pad fold, so no per-pixel intermediate besides one selection byte is stored.
#include "vfd_common.h"

namespace vfd {

constexpr int TS = 16;                  // tile side
constexpr float C1 = 0.0001f;           // 0.01 ** 2
constexpr float C2 = 0.0009f;           // 0.03 ** 2

// bt = blockIdx.z = b * cam_count + target slot (per-target arrays); br = b * N + cam (rig arrays)
struct PTarget {
  int bt, b, slot, cam;
  size_t br;
};
__device__ __forceinline__ PTarget ptarget_of(const vfd_photo_desc& d) {
  PTarget t;
  t.bt = blockIdx.z;
  t.b = t.bt / d.cam_count;
  t.slot = t.bt % d.cam_count;
  t.cam = d.cam_begin + t.slot;
  t.br = (size_t)t.b * d.N + t.cam;
  return t;
}

struct Moments {
  float mp, mt, spp, stt, spt;          // window means of p, t, p^2, t^2, p*t
};

// 3x3 window sums from an LDS plane with row pitch `pitch`, centre at (ly, lx).
__device__ __forceinline__ Moments window(const float* __restrict__ P, const float* __restrict__ Tt, int pitch,
                                          int ly, int lx) {
  float sp = 0.f, st = 0.f, spp = 0.f, stt = 0.f, spt = 0.f;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) {
      const float p = P[(ly + dy) * pitch + lx + dx];
      const float t = Tt[(ly + dy) * pitch + lx + dx];
      sp += p;
      st += t;
      spp += p * p;
      stt += t * t;
      spt += p * t;
    }
  return {sp / 9.f, st / 9.f, spp / 9.f, stt / 9.f, spt / 9.f};
}

__device__ __forceinline__ float ssim_of(const Moments& m) {
  const float mpt = m.mp * m.mt;
  const float mp2 = m.mp * m.mp, mt2 = m.mt * m.mt;
  const float sp = m.spp - mp2, st = m.stt - mt2, spt = m.spt - mpt;
  return ((2.f * mpt + C1) * (2.f * spt + C2)) / ((mp2 + mt2 + C1) * (sp + st + C2) + 1e-8f);
}

__device__ __forceinline__ float ssim_loss_of(const Moments& m) {
  return fminf(fmaxf((1.f - ssim_of(m)) / 2.f, 0.f), 1.f);
}

// ------------------------------------------------------------------------------ forward
// LDS planes (pitch TS+2): [0..2] target, then for each image slot 3 channel planes.
// image slots: 0..T-1 warped colour, T..2T-1 identity sources, 2T..2T+F-1 overlaps.
__global__ __launch_bounds__(256) void photo_fwd_k(vfd_photo_desc d, const float* __restrict__ target,
                                                   const float* __restrict__ color, const float* __restrict__ ovl,
                                                   const float* __restrict__ ref_mask,
                                                   const float* __restrict__ omask, const float* __restrict__ noise,
                                                   float* __restrict__ reproj, float* __restrict__ automask,
                                                   float* __restrict__ spatio_mask, uint8_t* __restrict__ sel,
                                                   double* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ double lds_red[4];
  constexpr int PT = TS + 2, PA = PT * PT;
  const int T = d.T, F = d.F;
  const int n_img = 2 * T + F;
  const PTarget tg = ptarget_of(d);
  const int bn = tg.bt, b = tg.b;
  const size_t br = tg.br;
  const int H = d.H, W = d.W, HW = H * W;
  const int ty0 = blockIdx.y * TS, tx0 = blockIdx.x * TS;
  // ---- stage tiles (+1 reflect halo)
  for (int i = threadIdx.x; i < PA; i += blockDim.x) {
    const int ly = i / PT, lx = i % PT;
    const int gy = min(reflect1(ty0 + ly - 1, H), H - 1), gx = min(reflect1(tx0 + lx - 1, W), W - 1);
    const size_t off = (size_t)gy * W + gx;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) smem[ch * PA + i] = target[(br * 3 + ch) * HW + off];
    for (int k = 0; k < n_img; ++k) {
      const float* src;
      if (k < T) src = color + (((size_t)bn * T + k) * 3) * HW;
      else if (k < 2 * T) src = d.ident[k - T] + (br * 3) * HW;
      else src = ovl + (((size_t)bn * F + (k - 2 * T)) * 3) * HW;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) smem[(3 + 3 * k + ch) * PA + i] = src[(size_t)ch * HW + off];
    }
  }
  __syncthreads();
  const int ly = threadIdx.x / TS + 1, lx = threadIdx.x % TS + 1;
  const int gy = ty0 + ly - 1, gx = tx0 + lx - 1;
  const bool inside = gy < H && gx < W;
  double acc[6] = {0, 0, 0, 0, 0, 0};
  if (inside) {
    const int p = gy * W + gx;
    const int c0 = ly * PT + lx;
    // photometric value of image slot k
    auto photo = [&](int k) {
      float ls = 0.f, l1 = 0.f;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        const float* P = smem + (3 + 3 * k + ch) * PA;
        const float* Tt = smem + ch * PA;
        ls += ssim_loss_of(window(P, Tt, PT, ly, lx));
        l1 += fabsf(Tt[c0] - P[c0]);
      }
      return 0.85f * (ls / 3.f) + 0.15f * (l1 / 3.f);
    };
    // reprojection: min over temporal warps, first index on ties
    float rep = 0.f;
    int ridx = 0;
    for (int f = 0; f < T; ++f) {
      const float v = photo(f);
      if (f == 0 || v < rep) { rep = v; ridx = f; }
    }
    float idn = 0.f;
    for (int f = 0; f < T; ++f) {
      const size_t ni = (((size_t)tg.slot * d.B + b) * T + f) * HW + p;
      const size_t hi = (((size_t)tg.cam * d.B + b) * T + f) * HW + p;
      const uint64_t seed = d.step ? d.seed ^ ((uint64_t)(*d.step) * 0x9E3779B97F4A7C15ULL) : d.seed;
      const float nz = noise ? d.noise_scale * noise[ni] : d.noise_scale * hash_normal(seed, hi);
      const float v = photo(T + f) + nz;
      if (f == 0 || v < idn) idn = v;
    }
    const bool auto_bit = !(idn < rep);                  // argmin([rep, idn]) == 0
    const float rm = ref_mask[br * HW + p];
    const float am = (auto_bit ? 1.f : 0.f) * rm;
    reproj[(size_t)bn * HW + p] = am * rep;
    automask[(size_t)bn * HW + p] = am;
    acc[0] = (double)(rep * am);
    acc[1] = (double)am;
    int sidx = 0;
    if (F > 0) {
      const float sm = rm * omask[((size_t)bn * F + 0) * HW + p];
      spatio_mask[(size_t)bn * HW + p] = sm;
      acc[2] = (double)(photo(2 * T) * sm);
      acc[3] = (double)sm;
      float st = 0.f, mst = 0.f;
      for (int f = 0; f < T; ++f) {
        const float v = photo(2 * T + 1 + f);
        if (f == 0 || v < st) { st = v; sidx = f; }
        const float pm = rm * omask[((size_t)bn * F + 1 + f) * HW + p] * am;
        mst = f == 0 ? pm : fmaxf(mst, pm);
      }
      acc[4] = (double)(st * mst);
      acc[5] = (double)mst;
    }
    sel[(size_t)bn * HW + p] = (uint8_t)(ridx | (auto_bit ? 4 : 0) | (sidx << 3));
  }
  const int nblk = gridDim.x * gridDim.y;
  const int blk = blockIdx.y * gridDim.x + blockIdx.x;
  double* out = partial + ((size_t)bn * nblk + blk) * 6;
  for (int i = 0; i < 6; ++i) {
    double v = wave_sum(acc[i]);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) lds_red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) out[i] = lds_red[0] + lds_red[1] + lds_red[2] + lds_red[3];
  }
}

__global__ __launch_bounds__(256) void photo_finalize_k(vfd_photo_desc d, const double* __restrict__ partial, int nblk,
                                                        double* __restrict__ sums, float* __restrict__ losses) {
  // one block per target camera: fp64 block reductions over batch x tiles
  __shared__ double lds[4];
  const int cam = blockIdx.x;
  const int rows = d.B * nblk;
  double s[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double acc = 0.0;
    for (int r = threadIdx.x; r < rows; r += blockDim.x) {
      const int b = r / nblk, k = r % nblk;
      acc += partial[(((size_t)b * d.cam_count + cam) * nblk + k) * 6 + i];
    }
    s[i] = block_sum_all(acc, lds);
  }
  if (threadIdx.x != 0) return;
  for (int i = 0; i < 6; ++i) sums[cam * 6 + i] = s[i];
  // compute_masked_loss: (loss * mask).sum() / (mask.sum() + 1e-8), fp32 like the reference
  losses[cam * 3 + 0] = (float)s[0] / ((float)s[1] + 1e-8f);
  losses[cam * 3 + 1] = (float)s[2] / ((float)s[3] + 1e-8f);
  losses[cam * 3 + 2] = (float)s[4] / ((float)s[5] + 1e-8f);
}

// ------------------------------------------------------------------------------ backward
// LDS: images with a +2 reflect halo (pitch TS+4): target + T colours + F overlaps (3 ch each);
// per-pixel masks with a +1 halo (pitch TS+2); coefficient planes of the current image.
__global__ __launch_bounds__(256) void photo_bwd_k(vfd_photo_desc d, const float* __restrict__ target,
                                                   const float* __restrict__ color, const float* __restrict__ ovl,
                                                   const float* __restrict__ ref_mask, const float* __restrict__ omask,
                                                   const uint8_t* __restrict__ sel, const float* __restrict__ gcoef,
                                                   float* __restrict__ d_color, float* __restrict__ d_ovl) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int QT = TS + 4, QA = QT * QT;      // image tiles, halo 2
  constexpr int MT = TS + 2, MA = MT * MT;      // mask / coefficient tiles, halo 1
  const int T = d.T, F = d.F;
  const int n_img = T + F;
  const PTarget tg = ptarget_of(d);
  const int bn = tg.bt, cam = tg.slot;
  const size_t br = tg.br;
  const int H = d.H, W = d.W, HW = H * W;
  const int ty0 = blockIdx.y * TS, tx0 = blockIdx.x * TS;
  float* img = smem;                                   // (1 + n_img) * 3 * QA
  float* mrm = img + (1 + n_img) * 3 * QA;             // ref mask       MA
  float* mom = mrm + MA;                               // overlap masks  F * MA
  float* msel = mom + F * MA;                          // selection      MA (as float)
  float* coef = msel + MA;                             // 9 * MA: (A, B, C) x 3 channels
  for (int i = threadIdx.x; i < QA; i += blockDim.x) {
    const int ly = i / QT, lx = i % QT;
    const int gy = min(max(reflect1(ty0 + ly - 2, H), 0), H - 1);
    const int gx = min(max(reflect1(tx0 + lx - 2, W), 0), W - 1);
    const size_t off = (size_t)gy * W + gx;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) img[ch * QA + i] = target[(br * 3 + ch) * HW + off];
    for (int k = 0; k < n_img; ++k) {
      const float* src = k < T ? color + (((size_t)bn * T + k) * 3) * HW : ovl + (((size_t)bn * F + (k - T)) * 3) * HW;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) img[(3 + 3 * k + ch) * QA + i] = src[(size_t)ch * HW + off];
    }
  }
  for (int i = threadIdx.x; i < MA; i += blockDim.x) {
    const int gy = ty0 + i / MT - 1, gx = tx0 + i % MT - 1;
    const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
    const size_t p = (size_t)gy * W + gx;
    mrm[i] = in ? ref_mask[br * HW + p] : 0.f;
    for (int s = 0; s < F; ++s) mom[s * MA + i] = in ? omask[((size_t)bn * F + s) * HW + p] : 0.f;
    msel[i] = in ? (float)sel[(size_t)bn * HW + p] : -1.f;
  }
  __syncthreads();
  const float gR = gcoef[cam * 3 + 0], gS = gcoef[cam * 3 + 1], gT = gcoef[cam * 3 + 2];
  const int qy = threadIdx.x / TS, qx = threadIdx.x % TS;      // output pixel in tile
  const int gy = ty0 + qy, gx = tx0 + qx;
  const bool inside = gy < H && gx < W;
  // row / column multisets of windows touching q, with the reflect fold
  int rows[5], cols[5], nr = 0, nc = 0;
  if (inside) {
    for (int dy = -1; dy <= 1; ++dy) if (gy + dy >= 0 && gy + dy < H) rows[nr++] = gy + dy;
    if (gy == 1) rows[nr++] = 0;
    if (gy == H - 2) rows[nr++] = H - 1;
    for (int dx = -1; dx <= 1; ++dx) if (gx + dx >= 0 && gx + dx < W) cols[nc++] = gx + dx;
    if (gx == 1) cols[nc++] = 0;
    if (gx == W - 2) cols[nc++] = W - 1;
  }
  for (int k = 0; k < n_img; ++k) {
    // ---- dL/dphoto at every output pixel of the +1 halo, then SSIM chain coefficients
    for (int i = threadIdx.x; i < MA; i += blockDim.x) {
      const int my = i / MT, mx = i % MT;
      float gph = 0.f;
      const float sv = msel[i];
      if (sv >= 0.f) {
        const int sb = (int)sv;
        const float rm = mrm[i];
        const float am = ((sb & 4) ? 1.f : 0.f) * rm;
        if (k < T) {
          if ((sb & 3) == k) gph = gR * am;
        } else if (k == T) {
          gph = gS * (rm * mom[i]);
        } else {
          const int f = k - T - 1;
          if (((sb >> 3) & 3) == f) {
            float mst = 0.f;
            for (int ff = 0; ff < T; ++ff) {
              const float pm = rm * mom[(1 + ff) * MA + i] * am;
              mst = ff == 0 ? pm : fmaxf(mst, pm);
            }
            gph = gT * mst;
          }
        }
      }
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        float A = 0.f, Bc = 0.f, Cc = 0.f;
        if (gph != 0.f) {
          const float* P = img + (3 + 3 * k + ch) * QA;
          const float* Tt = img + ch * QA;
          const Moments m = window(P, Tt, QT, my + 1, mx + 1);
          const float mpt = m.mp * m.mt, mp2 = m.mp * m.mp, mt2 = m.mt * m.mt;
          const float A1 = 2.f * mpt + C1, A2 = 2.f * (m.spt - mpt) + C2;
          const float B1 = mp2 + mt2 + C1, B2 = (m.spp - mp2) + (m.stt - mt2) + C2;
          const float Dn = B1 * B2 + 1e-8f;
          const float ssim = (A1 * A2) / Dn;
          const float lv = (1.f - ssim) / 2.f;
          if (lv >= 0.f && lv <= 1.f) {
            const float g = gph * (0.85f / 3.f) * -0.5f;
            A = g * ((2.f * m.mt * (A2 - A1)) / Dn - ssim * (2.f * m.mp * (B2 - B1)) / Dn);
            Bc = g * (-ssim * B1 / Dn);
            Cc = g * (2.f * A1 / Dn);
          }
        }
        coef[(ch * 3 + 0) * MA + i] = A;
        coef[(ch * 3 + 1) * MA + i] = Bc;
        coef[(ch * 3 + 2) * MA + i] = Cc;
      }
    }
    __syncthreads();
    if (inside) {
      const int ci = (qy + 2) * QT + qx + 2;
      const int mi = (qy + 1) * MT + qx + 1;
      // dL/dphoto at q itself for the L1 term
      float gq = 0.f;
      {
        const float sv = msel[mi];
        const int sb = (int)sv;
        const float rm = mrm[mi];
        const float am = ((sb & 4) ? 1.f : 0.f) * rm;
        if (k < T) {
          if ((sb & 3) == k) gq = gR * am;
        } else if (k == T) {
          gq = gS * (rm * mom[mi]);
        } else if (((sb >> 3) & 3) == k - T - 1) {
          float mst = 0.f;
          for (int ff = 0; ff < T; ++ff) {
            const float pm = rm * mom[(1 + ff) * MA + mi] * am;
            mst = ff == 0 ? pm : fmaxf(mst, pm);
          }
          gq = gT * mst;
        }
      }
      float* dst = k < T ? d_color + (((size_t)bn * T + k) * 3) * HW : d_ovl + (((size_t)bn * F + (k - T)) * 3) * HW;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        float sA = 0.f, sB = 0.f, sC = 0.f;
        for (int a = 0; a < nr; ++a)
          for (int c2 = 0; c2 < nc; ++c2) {
            const int m = (rows[a] - ty0 + 1) * MT + (cols[c2] - tx0 + 1);
            sA += coef[(ch * 3 + 0) * MA + m];
            sB += coef[(ch * 3 + 1) * MA + m];
            sC += coef[(ch * 3 + 2) * MA + m];
          }
        const float pv = img[(3 + 3 * k + ch) * QA + ci], tv = img[ch * QA + ci];
        float g = (sA + 2.f * pv * sB + tv * sC) / 9.f;
        const float diff = tv - pv;
        g += gq * (0.15f / 3.f) * (diff > 0.f ? -1.f : (diff < 0.f ? 1.f : 0.f));
        dst[(size_t)ch * HW + (size_t)gy * W + gx] = g;
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------ smoothness
constexpr int SBLK = 256, SPPT = 4;

__global__ __launch_bounds__(SBLK) void smooth_fwd_k(int B, int N, int H, int W, const float* __restrict__ disp,
                                                     const float* __restrict__ color, double* __restrict__ partial) {
  __shared__ double lds[4];
  const int bn = blockIdx.y, HW = H * W;
  const float* dp = disp + (size_t)bn * HW;
  const float* cl = color + (size_t)bn * 3 * HW;
  double s[3] = {0, 0, 0};
#pragma unroll
  for (int k = 0; k < SPPT; ++k) {
    const int p = blockIdx.x * SBLK * SPPT + k * SBLK + threadIdx.x;
    if (p >= HW) continue;
    const int x = p % W, y = p / W;
    const float dv = dp[p];
    s[0] += dv;
    if (x < W - 1) {
      const float gi = (fabsf(cl[p] - cl[p + 1]) + fabsf(cl[HW + p] - cl[HW + p + 1]) +
                        fabsf(cl[2 * HW + p] - cl[2 * HW + p + 1])) / 3.f;
      s[1] += (double)(fabsf(dv - dp[p + 1]) * expf(-1.f * gi));
    }
    if (y < H - 1) {
      const float gi = (fabsf(cl[p] - cl[p + W]) + fabsf(cl[HW + p] - cl[HW + p + W]) +
                        fabsf(cl[2 * HW + p] - cl[2 * HW + p + W])) / 3.f;
      s[2] += (double)(fabsf(dv - dp[p + W]) * expf(-1.f * gi));
    }
  }
  double* out = partial + ((size_t)bn * gridDim.x + blockIdx.x) * 3;
  for (int i = 0; i < 3; ++i) {
    double v = wave_sum(s[i]);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) out[i] = lds[0] + lds[1] + lds[2] + lds[3];
  }
}

__global__ __launch_bounds__(256) void smooth_finalize_k(int B, int N, int H, int W, const double* __restrict__ partial,
                                                         int nblk, double* __restrict__ sums, float* __restrict__ loss) {
  // one block per camera
  __shared__ double lds[4];
  const int cam = blockIdx.x;
  const double nx = (double)B * H * (W - 1), ny = (double)B * (H - 1) * W;
  double tot = 0.0;
  for (int b = 0; b < B; ++b) {
    const size_t bn = (size_t)b * N + cam;
    double s[3];
    for (int i = 0; i < 3; ++i) {
      double acc = 0.0;
      for (int k = threadIdx.x; k < nblk; k += blockDim.x) acc += partial[(bn * nblk + k) * 3 + i];
      s[i] = block_sum_all(acc, lds);
    }
    if (threadIdx.x == 0) {
      for (int i = 0; i < 3; ++i) sums[bn * 3 + i] = s[i];
      const double m = (double)(float)(s[0] / ((double)H * W)) + 1e-8;
      tot += s[1] / (m * nx) + s[2] / (m * ny);
    }
  }
  if (threadIdx.x == 0) loss[cam] = (float)tot;
}

__global__ __launch_bounds__(SBLK) void smooth_bwd_k(int B, int N, int H, int W, const float* __restrict__ disp,
                                                     const float* __restrict__ color, const double* __restrict__ sums,
                                                     const float* __restrict__ g, float* __restrict__ d_disp) {
  const int bn = blockIdx.y, HW = H * W, cam = bn % N;
  const int p = blockIdx.x * SBLK + threadIdx.x;
  if (p >= HW) return;
  const float* dp = disp + (size_t)bn * HW;
  const float* cl = color + (size_t)bn * 3 * HW;
  const double nx = (double)B * H * (W - 1), ny = (double)B * (H - 1) * W;
  const double* sm = sums + (size_t)bn * 3;
  const double m = (double)(float)(sm[0] / ((double)HW)) + 1e-8;
  const int x = p % W, y = p / W;
  auto edge = [&](int q0, int q1) {
    const float gi = (fabsf(cl[q0] - cl[q1]) + fabsf(cl[HW + q0] - cl[HW + q1]) + fabsf(cl[2 * HW + q0] - cl[2 * HW + q1])) / 3.f;
    return expf(-1.f * gi);
  };
  auto sgn = [](float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); };
  double G = 0.0;
  const float dv = dp[p];
  if (x < W - 1) G += (double)(edge(p, p + 1) * sgn(dv - dp[p + 1])) / nx;
  if (x > 0) G -= (double)(edge(p - 1, p) * sgn(dp[p - 1] - dv)) / nx;
  if (y < H - 1) G += (double)(edge(p, p + W) * sgn(dv - dp[p + W])) / ny;
  if (y > 0) G -= (double)(edge(p - W, p) * sgn(dp[p - W] - dv)) / ny;
  const double Fb = sm[1] / nx + sm[2] / ny;
  const double grad = G / m - Fb / (m * m * (double)HW);
  d_disp[(size_t)bn * HW + p] = (float)(grad * (double)g[cam]);
}

}  // namespace vfd

// ================================================================================== C ABI
using namespace vfd;

static int check_photo(const vfd_photo_desc* d) {
  VFD_REQUIRE(d != nullptr, "null descriptor");
  VFD_REQUIRE(d->B > 0 && d->N > 0 && d->H > 2 && d->W > 2, "bad photo sizes");
  VFD_REQUIRE(d->T >= 1 && d->T <= 3 && d->F >= 0 && d->F <= 4, "T=%d F=%d unsupported", d->T, d->F);
  VFD_REQUIRE(d->F == 0 || d->F == d->T + 1, "overlap slots must be 0 or T+1");
  VFD_REQUIRE(d->cam_count > 0 && d->cam_begin >= 0 && d->cam_begin + d->cam_count <= d->N, "bad target range");
  for (int f = 0; f < d->T; ++f) VFD_REQUIRE(d->ident[f] != nullptr, "identity source %d not set", f);
  return VFD_OK;
}

static dim3 photo_grid(const vfd_photo_desc* d) { return dim3(cdiv(d->W, TS), cdiv(d->H, TS), d->B * d->cam_count); }

extern "C" {

size_t vfd_photo_workspace_bytes(const vfd_photo_desc* d) {
  dim3 g = photo_grid(d);
  return (size_t)g.x * g.y * g.z * 6 * sizeof(double);
}

int vfd_photo_fwd(const vfd_photo_desc* d, const float* target, const float* color, const float* ovl,
                  const float* ref_mask, const float* omask, const float* noise, float* reproj, float* automask,
                  float* spatio_mask, uint8_t* sel, double* sums, float* losses, void* ws, size_t ws_bytes,
                  void* stream) {
  int st = check_photo(d);
  if (st) return st;
  VFD_REQUIRE(ws_bytes >= vfd_photo_workspace_bytes(d), "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  dim3 g = photo_grid(d);
  const int n_img = 2 * d->T + d->F;
  const size_t lds = (size_t)(3 + 3 * n_img) * (TS + 2) * (TS + 2) * sizeof(float);
  {
    ProfScope ps(K_PHOTO_FWD, s);
    photo_fwd_k<<<g, 256, lds, s>>>(*d, target, color, ovl, ref_mask, omask, noise, reproj, automask, spatio_mask,
                                     sel, (double*)ws);
  }
  if ((st = fail_launch("photo_fwd"))) return st;
  photo_finalize_k<<<d->cam_count, 256, 0, s>>>(*d, (const double*)ws, g.x * g.y, sums, losses);
  return fail_launch("photo_finalize");
}

int vfd_photo_bwd(const vfd_photo_desc* d, const float* target, const float* color, const float* ovl,
                  const float* ref_mask, const float* omask, const uint8_t* sel, const float* gcoef, float* d_color,
                  float* d_ovl, void* stream) {
  int st = check_photo(d);
  if (st) return st;
  hipStream_t s = (hipStream_t)stream;
  dim3 g = photo_grid(d);
  const int n_img = d->T + d->F;
  const int QA = (TS + 4) * (TS + 4), MA = (TS + 2) * (TS + 2);
  const size_t lds = ((size_t)(1 + n_img) * 3 * QA + (size_t)(2 + d->F) * MA + 9 * MA) * sizeof(float);
  ProfScope ps(K_PHOTO_BWD, s);
  photo_bwd_k<<<g, 256, lds, s>>>(*d, target, color, ovl, ref_mask, omask, sel, gcoef, d_color, d_ovl);
  return fail_launch("photo_bwd");
}

size_t vfd_smooth_workspace_bytes(int B, int N, int H, int W) {
  return (size_t)B * N * cdiv((size_t)H * W, SBLK * SPPT) * 3 * sizeof(double);
}

int vfd_smooth_fwd(int B, int N, int H, int W, const float* disp, const float* color, double* sums, float* loss,
                   void* ws, size_t ws_bytes, void* stream) {
  VFD_REQUIRE(B > 0 && N > 0 && H > 1 && W > 1, "bad smooth sizes");
  VFD_REQUIRE(ws_bytes >= vfd_smooth_workspace_bytes(B, N, H, W), "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const unsigned nblk = cdiv((size_t)H * W, SBLK * SPPT);
  {
    ProfScope ps(K_SMOOTH_FWD, s);
    smooth_fwd_k<<<dim3(nblk, B * N), SBLK, 0, s>>>(B, N, H, W, disp, color, (double*)ws);
  }
  int st = fail_launch("smooth_fwd");
  if (st) return st;
  smooth_finalize_k<<<N, 256, 0, s>>>(B, N, H, W, (const double*)ws, nblk, sums, loss);
  return fail_launch("smooth_finalize");
}

int vfd_smooth_bwd(int B, int N, int H, int W, const float* disp, const float* color, const double* sums,
                   const float* g, float* d_disp, void* stream) {
  VFD_REQUIRE(B > 0 && N > 0 && H > 1 && W > 1, "bad smooth sizes");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_SMOOTH_BWD, s);
  smooth_bwd_k<<<dim3(cdiv((size_t)H * W, SBLK), B * N), SBLK, 0, s>>>(B, N, H, W, disp, color, sums, g, d_disp);
  return fail_launch("smooth_bwd");
}

}  // extern "C"
