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
constexpr int PH_MAXI = 10;             // image slots 2T + F <= 2*3 + 4
constexpr float C1 = 0.0001f;           // 0.01 ** 2
constexpr float C2 = 0.0009f;           // 0.03 ** 2

// bt = blockIdx.z = b * cam_count + target slot (per-target arrays); br = b * N + cam (rig arrays)
struct PTarget {
  int bt, b, slot, cam;
  size_t br;
};
__device__ __forceinline__ PTarget ptarget_of(const vfd_photo_desc& d, int bz = -1) {
  PTarget t;
  t.bt = bz >= 0 ? bz : (int)blockIdx.z;
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
  __shared__ double lds_red[6][4];
  constexpr int PT = TS + 2, PA = PT * PT;
  const int T = d.T, F = d.F;
  const int n_img = 2 * T + F;
  // XCD-contiguous tiles: workgroups are dealt round-robin to the 8 XCDs, so the linear tile
  // index (L % 8) * (total / 8) + L / 8 hands each XCD a contiguous band of tile rows — a tile's
  // halo rows and the cache lines it shares with its neighbours are then fetched into the same
  // L2 once instead of once per XCD
  const uint3 bi = xcd_tile();
  const PTarget tg = ptarget_of(d, (int)bi.z);
  const int bn = tg.bt, b = tg.b;
  const size_t br = tg.br;
  const int H = d.H, W = d.W, HW = H * W;
  const int ty0 = bi.y * TS, tx0 = bi.x * TS;
  // ---- stage tiles (+1 reflect halo)
  // every plane's value of an LDS position is loaded before any is stored, so the 3 + 3 n_img
  // gathers of a thread are in flight together (a load -> store loop ran them as round trips)
  for (int i = threadIdx.x; i < PA; i += blockDim.x) {
    const int ly = i / PT, lx = i % PT;
    const int gy = min(reflect1(ty0 + ly - 1, H), H - 1), gx = min(reflect1(tx0 + lx - 1, W), W - 1);
    const size_t off = (size_t)gy * W + gx;
    float v[3 + 3 * PH_MAXI];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) v[ch] = target[(br * 3 + ch) * HW + off];
#pragma unroll
    for (int k = 0; k < PH_MAXI; ++k) {
      const int kk = k < n_img ? k : 0;
      const float* src;
      if (kk < T) src = color + (((size_t)bn * T + kk) * 3) * HW;
      else if (kk < 2 * T) src = d.ident[kk - T] + (br * 3) * HW;
      else src = ovl + (((size_t)bn * F + (kk - 2 * T)) * 3) * HW;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) v[3 + 3 * k + ch] = src[(size_t)ch * HW + off];
    }
#pragma unroll
    for (int k = 0; k < 3 + 3 * PH_MAXI; ++k)
      if (k < 3 + 3 * n_img) smem[k * PA + i] = v[k];
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
  const int blk = bi.y * gridDim.x + bi.x;
  double* out = partial + ((size_t)bn * nblk + blk) * 6;
  // the six block sums in one round (same wave sums, same wave order as one round per sum)
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const double v = wave_sum(acc[i]);
    if ((threadIdx.x & 63) == 0) lds_red[i][threadIdx.x >> 6] = v;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    const double* r = lds_red[threadIdx.x];
    out[threadIdx.x] = r[0] + r[1] + r[2] + r[3];
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
// Register sliding window, no LDS: a wave owns one image k and a strip of 64 columns (60 output
// columns + a 2-column halo each side) x PB_R rows and walks it top to bottom, one input row per
// step: lanes = columns (coalesced row loads), horizontal neighbours by lane shuffles, the last
// three rows of window sums / coefficient sums kept in registers (ring unrolled by 3).
//   step i: load row i (reflect-padded) -> horizontal 3-sums of (p, t, pp, tt, pt);
//           window at m = i-1 -> SSIM chain coefficients (A, B, C) * dL/dphoto(m), summed over
//           the transposed horizontal window (x2 on the reflect-folded neighbour);
//           gradient at q = i-2 = vertical transposed sum (A + 2 p B + t C) / 9 + L1 term.
// The transposed window sums carry the reflect fold: the neighbour term counts twice at
// q == 1 and q == n-2 (loss_util.py:43-67 pads by reflection before the 3x3 pools).
constexpr int PB_R = 32;        // output rows per strip
constexpr int PB_OC = 60;       // output columns per wave

// lane L <- lane L-1 / L+1 of the wave (DPP wave_shr:1 / wave_shl:1: a VALU modifier, no LDS);
// the end lanes receive 0 (they only feed halo lanes)
__device__ __forceinline__ float from_left(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ float from_right(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xF, 0xF, false));
}

struct PRow {
  float hm[3][5];               // horizontal window sums of p, t, p^2, t^2, p*t per channel
  float cf[3][3];               // transposed horizontal sums of A, B, C per channel
  float p[3], t[3];             // the pixel's own values
  float g;                      // dL/dphoto at the pixel
};

__global__ __launch_bounds__(256) void photo_bwd_k(vfd_photo_desc d, const float* __restrict__ target,
                                                   const float* __restrict__ color, const float* __restrict__ ovl,
                                                   const float* __restrict__ ref_mask, const float* __restrict__ omask,
                                                   const uint8_t* __restrict__ sel, const float* __restrict__ gcoef,
                                                   float* __restrict__ d_color, float* __restrict__ d_ovl) {
  const int T = d.T, F = d.F;
  const int n_img = T + F;
  const PTarget tg = ptarget_of(d);
  const int bn = tg.bt, cam = tg.slot;
  const size_t br = tg.br;
  const int H = d.H, W = d.W, HW = H * W;
  const int nsx = (W + PB_OC - 1) / PB_OC, nsy = (H + PB_R - 1) / PB_R;
  const int task = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= n_img * nsx * nsy) return;                 // whole wave; no barriers below
  const int k = task % n_img, sx = (task / n_img) % nsx, sy = task / (n_img * nsx);
  const int lane = threadIdx.x & 63;
  const int c = sx * PB_OC - 2 + lane;
  const bool col_in = c >= 0 && c < W;
  const bool out_lane = lane >= 2 && lane < 2 + PB_OC && col_in;
  const int cr = min(max(c < 0 ? -c : (c > W - 1 ? 2 * (W - 1) - c : c), 0), W - 1);
  const int cc = min(max(c, 0), W - 1);                  // clamped real column (masks)
  const int r0 = sy * PB_R, r1 = min(r0 + PB_R, H);
  const float* P = k < T ? color + (((size_t)bn * T + k) * 3) * HW : ovl + (((size_t)bn * F + (k - T)) * 3) * HW;
  const float* Tg = target + br * 3 * HW;
  float* dst = k < T ? d_color + (((size_t)bn * T + k) * 3) * HW : d_ovl + (((size_t)bn * F + (k - T)) * 3) * HW;
  const float gR = gcoef[cam * 3 + 0], gS = gcoef[cam * 3 + 1], gT = gcoef[cam * 3 + 2];
  const float wl = c == 1 ? 2.f : 1.f, wr = c == W - 2 ? 2.f : 1.f;
  const uint8_t* selb = sel + (size_t)bn * HW;
  const float* rmb = ref_mask + br * HW;
  const float* omb = omask + (size_t)bn * F * HW;

  // All loads of a step (image row i, mask row i - 1) are unconditional at clamped addresses and
  // sit in one basic block ahead of the arithmetic, so they are one memory round trip together
  // (behind the row / selection branches they were three dependent ones, and a wave walks ~36 rows
  // in sequence with only a few waves per SIMD to hide it).
  const float* omp = F > 0 ? omb : rmb;                  // any readable plane when F == 0 (k < T)
  auto step = [&](int i, PRow& nw, PRow& o1, PRow& o2) {
    if (i > r1 + 1) return;
    const int m = i - 1;
    const size_t pm = (size_t)min(max(m, 0), H - 1) * W + cc;
    const int sb = selb[pm];
    const float rm = rmb[pm];
    float om[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) om[j] = omp[(size_t)(F > 0 ? min(k == T ? 0 : 1 + j, F - 1) : 0) * HW + pm];
    const int ri = min(max(i < 0 ? -i : (i > H - 1 ? 2 * (H - 1) - i : i), 0), H - 1);
    const size_t roff = (size_t)ri * W + cr;
    float pr_[3], tr_[3];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      pr_[ch] = P[(size_t)ch * HW + roff];
      tr_[ch] = Tg[(size_t)ch * HW + roff];
    }
    // keep the loads here (the optimiser would sink each into the branch that reads it)
    asm volatile("" ::"v"(sb), "v"(rm), "v"(om[0]), "v"(om[1]), "v"(om[2]));
    asm volatile("" ::"v"(pr_[0]), "v"(pr_[1]), "v"(pr_[2]), "v"(tr_[0]), "v"(tr_[1]), "v"(tr_[2]));
    // dL/dphoto_k at real pixel (m, c) (0 outside the map)
    float gph = 0.f;
    if (m >= 0 && m < H && col_in) {
      const float am = ((sb & 4) ? 1.f : 0.f) * rm;
      if (k < T) {
        if ((sb & 3) == k) gph = gR * am;
      } else if (k == T) {
        gph = gS * (rm * om[0]);
      } else if (((sb >> 3) & 3) == k - T - 1) {
        float mst = 0.f;
#pragma unroll
        for (int ff = 0; ff < 3; ++ff) {
          if (ff >= T) break;
          const float pmv = rm * om[ff] * am;
          mst = ff == 0 ? pmv : fmaxf(mst, pmv);
        }
        gph = gT * mst;
      }
    }
    // ---- (1) input row i of the reflect-padded images
    if (i >= -1 && i <= H) {
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        const float p = pr_[ch], tv = tr_[ch];
        nw.p[ch] = p;
        nw.t[ch] = tv;
        const float pl = from_left(p), pr = from_right(p);
        const float tl = from_left(tv), tr = from_right(tv);
        nw.hm[ch][0] = pl + p + pr;
        nw.hm[ch][1] = tl + tv + tr;
        nw.hm[ch][2] = pl * pl + p * p + pr * pr;
        nw.hm[ch][3] = tl * tl + tv * tv + tr * tr;
        nw.hm[ch][4] = pl * tl + p * tv + pr * tr;
      }
    } else {
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        nw.p[ch] = nw.t[ch] = 0.f;
#pragma unroll
        for (int q = 0; q < 5; ++q) nw.hm[ch][q] = 0.f;
      }
    }
    // ---- (2) window centred at m = i - 1 -> coefficient sums of row m (slot o1)
    {
      o1.g = gph;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        float A = 0.f, Bc = 0.f, Cc = 0.f;
        if (gph != 0.f) {
          // window means: sums * (1/9) (the backward's arithmetic need not repeat the forward's
          // division; the clamp test below sits on ssim, far from rounding at +-1)
          constexpr float inv9 = 1.f / 9.f;
          const float mp = (o2.hm[ch][0] + o1.hm[ch][0] + nw.hm[ch][0]) * inv9;
          const float mt = (o2.hm[ch][1] + o1.hm[ch][1] + nw.hm[ch][1]) * inv9;
          const float spp = (o2.hm[ch][2] + o1.hm[ch][2] + nw.hm[ch][2]) * inv9;
          const float stt = (o2.hm[ch][3] + o1.hm[ch][3] + nw.hm[ch][3]) * inv9;
          const float spt = (o2.hm[ch][4] + o1.hm[ch][4] + nw.hm[ch][4]) * inv9;
          const float mpt = mp * mt, mp2 = mp * mp, mt2 = mt * mt;
          const float A1 = 2.f * mpt + C1, A2 = 2.f * (spt - mpt) + C2;
          const float B1 = mp2 + mt2 + C1, B2 = (spp - mp2) + (stt - mt2) + C2;
          const float rDn = 1.f / (B1 * B2 + 1e-8f);
          const float ssim = (A1 * A2) * rDn;
          const float lv = (1.f - ssim) * 0.5f;
          if (lv >= 0.f && lv <= 1.f) {
            const float g = gph * (0.85f / 3.f) * -0.5f * rDn;
            A = g * (2.f * mt * (A2 - A1) - ssim * (2.f * mp * (B2 - B1)));
            Bc = g * (-ssim * B1);
            Cc = g * (2.f * A1);
          }
        }
        o1.cf[ch][0] = from_left(A) * wl + A + from_right(A) * wr;
        o1.cf[ch][1] = from_left(Bc) * wl + Bc + from_right(Bc) * wr;
        o1.cf[ch][2] = from_left(Cc) * wl + Cc + from_right(Cc) * wr;
      }
    }
    // ---- (3) gradient at real row q = i - 2: rows q-1 (slot nw, not yet reused), q (o2), q+1 (o1)
    const int q = i - 2;
    if (q >= r0 && q < r1) {
      const float vl = q == 1 ? 2.f : 1.f, vr = q == H - 2 ? 2.f : 1.f;
      const size_t off = (size_t)q * W + cc;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        const float sA = nw.cf[ch][0] * vl + o2.cf[ch][0] + o1.cf[ch][0] * vr;
        const float sB = nw.cf[ch][1] * vl + o2.cf[ch][1] + o1.cf[ch][1] * vr;
        const float sC = nw.cf[ch][2] * vl + o2.cf[ch][2] + o1.cf[ch][2] * vr;
        const float pv = o2.p[ch], tv = o2.t[ch];
        float g = (sA + 2.f * pv * sB + tv * sC) * (1.f / 9.f);
        const float diff = tv - pv;
        g += o2.g * (0.15f / 3.f) * (diff > 0.f ? -1.f : (diff < 0.f ? 1.f : 0.f));
        if (out_lane) dst[(size_t)ch * HW + off] = g;
      }
    }
  };

  PRow R0, R1, R2;
  for (PRow* r : {&R0, &R1, &R2}) {
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
#pragma unroll
      for (int q = 0; q < 5; ++q) r->hm[ch][q] = 0.f;
#pragma unroll
      for (int q = 0; q < 3; ++q) r->cf[ch][q] = 0.f;
      r->p[ch] = r->t[ch] = 0.f;
    }
    r->g = 0.f;
  }
  for (int i = r0 - 2; i <= r1 + 1; i += 3) {
    step(i, R0, R2, R1);
    step(i + 1, R1, R0, R2);
    step(i + 2, R2, R1, R0);
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
  ProfScope ps(K_PHOTO_FWD, s);              // the op: maps + block partials + their reduction
  photo_fwd_k<<<g, 256, lds, s>>>(*d, target, color, ovl, ref_mask, omask, noise, reproj, automask, spatio_mask,
                                   sel, (double*)ws);
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
  const int n_img = d->T + d->F;
  const int ntask = n_img * cdiv(d->W, PB_OC) * cdiv(d->H, PB_R);
  ProfScope ps(K_PHOTO_BWD, s);
  photo_bwd_k<<<dim3(cdiv(ntask, 4), 1, d->B * d->cam_count), 256, 0, s>>>(*d, target, color, ovl, ref_mask, omask, sel,
                                                                       gcoef, d_color, d_ovl);
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
  ProfScope ps(K_SMOOTH_FWD, s);             // the op: block partials + their reduction
  smooth_fwd_k<<<dim3(nblk, B * N), SBLK, 0, s>>>(B, N, H, W, disp, color, (double*)ws);
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
