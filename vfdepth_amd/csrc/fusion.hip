// Volumetric fusion kernels for gfx950 (reference: network/volumetric_fusionnet.py).
//
//  mask_downsample    F.interpolate(mask, [h,w], bilinear, align_corners=True)          (:129)
//  K1 fuse_depth      unproject -> bilinear gather -> overlap/non-overlap 1x1 MLP -> LReLU
//                     -> count masks, voxel-major output [B,V,Cv]                   (:116-230)
//  K2 fuse_pose       unproject -> bilinear gather -> mean over valid cameras, written in
//                     the (reflect-padded) NCHW layout the stride-2 conv reads        (:116-162)
//  K3 voxel_project   frustum points -> trilinear gather of [B,V,Cv] -> [B*N,Cv*D,h,w]
//                     (reflect-padded for the 3x3 conv)                             (:232-262)
//
// Geometry (voxel<->camera) is recomputed in every kernel from K / E (a few dozen FLOPs per
// point) instead of being stored: it costs no HBM traffic and keeps forward and backward
// decisions bit-identical.  All arithmetic follows the reference's operation order with
// -ffp-contract=off so that validity tests at the boundaries agree with the CPU reference.
#include <algorithm>
#include <type_traits>

#include "vfd_common.h"

namespace vfd {

// ------------------------------------------------------------------------------ geometry
struct VoxCam {
  float ix, iy;   // unnormalised sample position in the h x w map (ATen align_corners=True)
  float z;        // camera-frame depth of the voxel centre
  bool valid;     // in front, inside the image, not self-occluded
};

// volumetric_fusionnet.py:132-140, 166-195, in two steps so a caller looping over the cameras can
// put every camera's mask load in flight before it tests any: voxel_project (arithmetic only, the
// nearest mask index) and voxel_finish (the validity test on the loaded mask value).
struct VoxProj {
  float ix, iy, z;
  int ni;         // nearest mask index, -1 when out of range / non-finite
  bool fin, oob;
};

__device__ __forceinline__ VoxProj voxel_project(const float* __restrict__ Kc, const float* __restrict__ Ei,
                                                 float x, float y, float z, int h, int w) {
  const float l0 = Ei[0] * x + Ei[1] * y + Ei[2] * z + Ei[3];
  const float l1 = Ei[4] * x + Ei[5] * y + Ei[6] * z + Ei[7];
  const float l2 = Ei[8] * x + Ei[9] * y + Ei[10] * z + Ei[11];
  const float c0 = Kc[0] * l0 + Kc[1] * l1 + Kc[2] * l2;
  const float c1 = Kc[4] * l0 + Kc[5] * l1 + Kc[6] * l2;
  const float c2 = Kc[8] * l0 + Kc[9] * l1 + Kc[10] * l2;
  const float den = c2 + 1e-8f;
  const float u = c0 / den, v = c1 / den;
  VoxProj p;
  p.z = l2;
  p.fin = finitef(u) && finitef(v);
  const float gx = (u / (float)(w - 1) - 0.5f) * 2.f;
  const float gy = (v / (float)(h - 1) - 0.5f) * 2.f;
  p.ix = unnorm_ac(gx, w);
  p.iy = unnorm_ac(gy, h);
  p.oob = (gx > 1.f) || (gx < -1.f) || (gy > 1.f) || (gy < -1.f);
  p.ni = p.fin ? nearest_index(p.ix, p.iy, w, h) : -1;
  return p;
}

// mask index to load for a projection (element 0 when there is none; voxel_finish drops it)
__device__ __forceinline__ int voxel_mask_index(const VoxProj& p) { return p.ni >= 0 ? p.ni : 0; }

__device__ __forceinline__ VoxCam voxel_finish(const VoxProj& p, float occ_raw) {
  VoxCam r;
  r.z = p.z;
  const float occ = p.ni >= 0 ? occ_raw : 0.f;
  // non-finite: the reference clamps to +-2w (always out of range) or propagates NaN; both -> invalid
  r.ix = p.fin ? p.ix : -1e9f;
  r.iy = p.fin ? p.iy : -1e9f;
  r.valid = p.fin && (occ > 0.5f) && (p.z > 0.f) && !p.oob;
  return r;
}

__device__ __forceinline__ VoxCam voxel_to_camera(const float* __restrict__ Kc, const float* __restrict__ Ei,
                                                  float x, float y, float z,
                                                  const float* __restrict__ mlo, int h, int w) {
  const VoxProj p = voxel_project(Kc, Ei, x, y, z, h, w);
  return voxel_finish(p, mlo[voxel_mask_index(p)]);
}

// A valid (voxel, camera) pair as the gather/scatter loops need it.
struct Tap {
  int cam;
  int base;        // y0 * w + x0
  float w[4];      // ATen corner weights, 0 for out-of-range corners
  unsigned in;     // in-range bit per corner (nw, ne, sw, se)
  float z;
};

__device__ __forceinline__ Tap make_tap(int cam, const VoxCam& g, int h, int w) {
  Bilinear b = bilinear_taps(g.ix, g.iy, w, h);
  Tap t;
  t.cam = cam;
  t.base = b.y0 * w + b.x0;
  t.in = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    t.w[k] = b.in[k] ? b.w[k] : 0.f;
    t.in |= (b.in[k] ? 1u : 0u) << k;
  }
  t.z = g.z;
  return t;
}

__device__ __forceinline__ int tap_offset(int k, int w) { return (k & 1) + (k >> 1) * w; }

__device__ __forceinline__ int rdl(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ float rdlf(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ unsigned rdlu(unsigned v, int lane) {
  return (unsigned)__builtin_amdgcn_readlane((int)v, lane);
}

// ------------------------------------------------------------------------------ mask downsample
__global__ void mask_downsample_k(const float* __restrict__ src, float* __restrict__ dst,
                                  int BN, int H, int W, int h, int w) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= BN * h * w) return;
  int x = i % w, y = (i / w) % h, n = i / (w * h);
  const float* s = src + (size_t)n * H * W;
  float sy = h > 1 ? (float)(H - 1) / (float)(h - 1) : 0.f;
  float sx = w > 1 ? (float)(W - 1) / (float)(w - 1) : 0.f;
  int y0, x0, y1, x1;
  float ly, lx;
  if (h == H) { y0 = y1 = y; ly = 0.f; } else {
    float fy = sy * (float)y;
    y0 = min((int)floorf(fy), H - 1);
    ly = fminf(fmaxf(fy - (float)y0, 0.f), 1.f);
    y1 = y0 + (y0 < H - 1 ? 1 : 0);
  }
  if (w == W) { x0 = x1 = x; lx = 0.f; } else {
    float fx = sx * (float)x;
    x0 = min((int)floorf(fx), W - 1);
    lx = fminf(fmaxf(fx - (float)x0, 0.f), 1.f);
    x1 = x0 + (x0 < W - 1 ? 1 : 0);
  }
  float h0 = 1.f - ly, w0 = 1.f - lx;
  float top = w0 * s[y0 * W + x0] + lx * s[y0 * W + x1];
  float bot = w0 * s[y1 * W + x0] + lx * s[y1 * W + x1];
  dst[i] = h0 * top + ly * bot;
}

// ------------------------------------------------------------------------------ K1 forward
// One wave owns 64 consecutive voxels.  Phase 1: lane i resolves voxel i's cameras.  Phase 2:
// the wave walks the 64 voxels; for each, every lane produces one output channel from the
// folded per-camera maps P (pixel-major rows of 2*Cv floats: 256-B coalesced tap reads).
template <int CPL>
__global__ __launch_bounds__(256) void fuse_depth_fwd_k(vfd_voxel_desc d, const float* __restrict__ P,
                                                        const float* __restrict__ mlo,
                                                        const float* __restrict__ K,
                                                        const float* __restrict__ Einv,
                                                        const float* __restrict__ wz,
                                                        const float* __restrict__ b_no,
                                                        const float* __restrict__ b_o,
                                                        float* __restrict__ vox) {
  const int lane = threadIdx.x & 63;
  const int V = d.X * d.Y * d.Z;
  const int b = blockIdx.y;
  const int v0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
  if (v0 >= V) return;
  const int hw = d.h * d.w;
  const int v = v0 + lane;
  int cnt = 0;
  Tap t0{}, t1{};
  if (v < V) {
    float x = d.axis_x[v % d.X], y = d.axis_y[(v / d.X) % d.Y], z = d.axis_z[v / (d.X * d.Y)];
    for (int c = 0; c < d.N; ++c) {
      const int bc = b * d.N + c;
      VoxCam g = voxel_to_camera(K + bc * 16, Einv + bc * 16, x, y, z, mlo + (size_t)bc * hw, d.h, d.w);
      if (g.valid) {
        if (cnt == 0) t0 = make_tap(c, g, d.h, d.w);
        else if (cnt == 1) t1 = make_tap(c, g, d.h, d.w);
        ++cnt;
      }
    }
  }
  const int twoCv = 2 * d.Cv;
  const int nvox = min(64, V - v0);
  float wzr[CPL][3], bno[CPL], bo[CPL];
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    int ch = lane + 64 * k;
    bool on = ch < d.Cv;
    wzr[k][0] = on ? wz[ch] : 0.f;
    wzr[k][1] = on ? wz[d.Cv + ch] : 0.f;
    wzr[k][2] = on ? wz[2 * d.Cv + ch] : 0.f;
    bno[k] = on ? b_no[ch] : 0.f;
    bo[k] = on ? b_o[ch] : 0.f;
  }
  for (int j = 0; j < nvox; ++j) {
    const int cj = rdl(cnt, j);
    float* out = vox + ((size_t)b * V + v0 + j) * d.Cv;
    if (cj != 1 && cj != 2) {
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        int ch = lane + 64 * k;
        if (ch < d.Cv) out[ch] = 0.f;
      }
      continue;
    }
    const int off = (cj == 1) ? 0 : d.Cv;
    float acc[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) acc[k] = 0.f;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (s >= cj) break;
      const Tap& tl = s == 0 ? t0 : t1;
      const int cam = rdl(tl.cam, j);
      const int base = rdl(tl.base, j);
      const unsigned in = rdlu(tl.in, j);
      const float zt = rdlf(tl.z, j);
      const float* Pc = P + (size_t)(b * d.N + cam) * hw * twoCv + off;
      float val[CPL];
#pragma unroll
      for (int k = 0; k < CPL; ++k) val[k] = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (!(in >> q & 1u)) continue;
        const float wq = rdlf(tl.w[q], j);
        const float* row = Pc + (size_t)(base + tap_offset(q, d.w)) * twoCv;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
          int ch = lane + 64 * k;
          if (ch < d.Cv) val[k] += row[ch] * wq;
        }
      }
      const int zrow = (cj == 1) ? 0 : 1 + d.group[cam];
#pragma unroll
      for (int k = 0; k < CPL; ++k) acc[k] += val[k] + wzr[k][zrow] * (zt / d.z_scale);
    }
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      int ch = lane + 64 * k;
      if (ch < d.Cv) {
        float pre = acc[k] + (cj == 1 ? bno[k] : bo[k]);
        out[ch] = pre > 0.f ? pre : pre * 0.1f;
      }
    }
  }
}

// Latency-tolerant variant for Cv in {16, 32, 64}: phase 1 (lane = voxel) writes each voxel's
// taps to LDS; phase 2 runs lanes = (voxel, channel quad), 64 / (Cv/4) voxels per instruction,
// branch-free: every voxel issues its 8 float4 corner reads (out-of-range corners and the missing
// second tap read a valid row with weight 0, which adds +0: the same per-channel operation
// sequence as fuse_depth_fwd_k), so two groups of voxels have all their loads in flight.
struct VoxRec {
  int cnt, cam[2], base[2];
  float w[2][4], z[2];
};

template <int CV>
__global__ __launch_bounds__(256) void fuse_depth_fwd_q_k(vfd_voxel_desc d, const float* __restrict__ P,
                                                          const float* __restrict__ mlo,
                                                          const float* __restrict__ K,
                                                          const float* __restrict__ Einv,
                                                          const float* __restrict__ wz,
                                                          const float* __restrict__ b_no,
                                                          const float* __restrict__ b_o,
                                                          float* __restrict__ vox) {
  constexpr int QPV = CV / 4, VPI = 64 / QPV;      // quads per voxel, voxels per instruction
  __shared__ VoxRec rec_l[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int V = d.X * d.Y * d.Z;
  const int b = blockIdx.y;
  const int v0 = (blockIdx.x * 4 + wv) * 64;
  if (v0 >= V) return;                               // whole wave; the block has no barrier
  const int hw = d.h * d.w;
  {
    const int v = v0 + lane;
    VoxRec r;
    r.cnt = 0;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      r.cam[s] = 0;
      r.base[s] = 0;
      r.z[s] = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) r.w[s][q] = 0.f;
    }
    if (v < V) {
      const float x = d.axis_x[v % d.X], y = d.axis_y[(v / d.X) % d.Y], z = d.axis_z[v / (d.X * d.Y)];
      for (int c = 0; c < d.N; ++c) {
        const int bc = b * d.N + c;
        VoxCam g = voxel_to_camera(K + bc * 16, Einv + bc * 16, x, y, z, mlo + (size_t)bc * hw, d.h, d.w);
        if (g.valid) {
          // (explicit slots: a runtime slot index would put the record in scratch)
          if (r.cnt == 0) {
            const Tap tp = make_tap(c, g, d.h, d.w);
            r.cam[0] = r.cam[1] = c;          // slot 1 defaults to a valid row (weight 0)
            r.base[0] = r.base[1] = tp.base;
            r.z[0] = tp.z;
#pragma unroll
            for (int q = 0; q < 4; ++q) r.w[0][q] = tp.w[q];
          } else if (r.cnt == 1) {
            const Tap tp = make_tap(c, g, d.h, d.w);
            r.cam[1] = c;
            r.base[1] = tp.base;
            r.z[1] = tp.z;
#pragma unroll
            for (int q = 0; q < 4; ++q) r.w[1][q] = tp.w[q];
          }
          ++r.cnt;
        }
      }
    }
    rec_l[wv][lane] = r;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0xc07f);                // lgkmcnt(0): the wave's LDS records are visible
  const int g = lane / QPV, q4 = lane % QPV;
  const int ch0 = q4 * 4;
  const float4 bno = *reinterpret_cast<const float4*>(b_no + ch0);
  const float4 bo = *reinterpret_cast<const float4*>(b_o + ch0);
  const float4 wz0 = *reinterpret_cast<const float4*>(wz + ch0);
  const float4 wz1 = *reinterpret_cast<const float4*>(wz + CV + ch0);
  const float4 wz2 = *reinterpret_cast<const float4*>(wz + 2 * CV + ch0);
  const int twoCv = 2 * CV;
  const int nvox = min(64, V - v0);
  for (int j0 = 0; j0 < nvox; j0 += VPI) {
    const int j = j0 + g;
    const VoxRec& r = rec_l[wv][min(j, 63)];
    const int cnt = j < nvox ? r.cnt : 0;
    const bool live = cnt == 1 || cnt == 2;
    const int off = cnt == 2 ? CV : 0;
    float4 v[2][4];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int cam = r.cam[s];
      const float* Pc = P + (size_t)(b * d.N + cam) * hw * twoCv + off + ch0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int pix = min(max(r.base[s] + tap_offset(q, d.w), 0), hw - 1);
        v[s][q] = *reinterpret_cast<const float4*>(Pc + (size_t)pix * twoCv);
      }
    }
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bool tap = s < cnt && live;
      float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float wq = tap ? r.w[s][q] : 0.f;
        val.x += v[s][q].x * wq;
        val.y += v[s][q].y * wq;
        val.z += v[s][q].z * wq;
        val.w += v[s][q].w * wq;
      }
      const int zrow = (cnt == 1) ? 0 : 1 + d.group[r.cam[s]];
      const float4 wzr = zrow == 0 ? wz0 : (zrow == 1 ? wz1 : wz2);
      const float zf = tap ? r.z[s] / d.z_scale : 0.f;
      if (tap) {
        acc.x += val.x + wzr.x * zf;
        acc.y += val.y + wzr.y * zf;
        acc.z += val.z + wzr.z * zf;
        acc.w += val.w + wzr.w * zf;
      }
    }
    const float4 bb = cnt == 1 ? bno : bo;
    float4 o;
    o.x = acc.x + bb.x;
    o.y = acc.y + bb.y;
    o.z = acc.z + bb.z;
    o.w = acc.w + bb.w;
    o.x = live ? (o.x > 0.f ? o.x : o.x * 0.1f) : 0.f;
    o.y = live ? (o.y > 0.f ? o.y : o.y * 0.1f) : 0.f;
    o.z = live ? (o.z > 0.f ? o.z : o.z * 0.1f) : 0.f;
    o.w = live ? (o.w > 0.f ? o.w : o.w * 0.1f) : 0.f;
    if (j < nvox) *reinterpret_cast<float4*>(vox + ((size_t)b * V + v0 + j) * CV + ch0) = o;
  }
}

// ------------------------------------------------------------------------------ K1 backward
// Same voxel walk; lanes are channels, so every scatter into dP is a 256-B contiguous row of
// f32 atomics (the full-rate atomic shape on gfx950).  Depth-column and bias gradients are
// reduced per lane and written as per-wave partials (summed by fuse_depth_reduce_k).
template <int CPL, bool SCATTER>
__global__ __launch_bounds__(256) void fuse_depth_bwd_k(vfd_voxel_desc d, const float* __restrict__ dvox,
                                                        const float* __restrict__ vox,
                                                        const float* __restrict__ mlo,
                                                        const float* __restrict__ K,
                                                        const float* __restrict__ Einv,
                                                        float* __restrict__ dP,
                                                        float* __restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const int V = d.X * d.Y * d.Z;
  const int b = blockIdx.y;
  const int wave_id = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int v0 = wave_id * 64;
  const int n_waves = (V + 63) / 64;
  float* part = partial + ((size_t)b * n_waves + wave_id) * 5 * d.Cv;
  float red[CPL][5];
#pragma unroll
  for (int k = 0; k < CPL; ++k)
#pragma unroll
    for (int r = 0; r < 5; ++r) red[k][r] = 0.f;
  if (v0 < V) {
    const int hw = d.h * d.w;
    const int v = v0 + lane;
    int cnt = 0;
    Tap t0{}, t1{};
    if (v < V) {
      float x = d.axis_x[v % d.X], y = d.axis_y[(v / d.X) % d.Y], z = d.axis_z[v / (d.X * d.Y)];
      for (int c = 0; c < d.N; ++c) {
        const int bc = b * d.N + c;
        VoxCam g = voxel_to_camera(K + bc * 16, Einv + bc * 16, x, y, z, mlo + (size_t)bc * hw, d.h, d.w);
        if (g.valid) {
          if (cnt == 0) t0 = make_tap(c, g, d.h, d.w);
          else if (cnt == 1) t1 = make_tap(c, g, d.h, d.w);
          ++cnt;
        }
      }
    }
    const int twoCv = 2 * d.Cv;
    const int nvox = min(64, V - v0);
    // Run merging: consecutive voxels of the walk whose camera slot hits the same (camera, column
    // half) footprint, or one shifted by one pixel along the row, add their weighted gradients in
    // registers; atomics are issued only for tap rows that leave the footprint.
    float racc[2][4][CPL];
    int rside[2] = {-1, -1};         // wave-uniform run state per camera slot: (column half, camera),
    int rbase[2] = {0, 0};           // -1 = no open run; base pixel (may be negative at the border)
    unsigned rin[2] = {0u, 0u};
    float* rrow[2] = {dP, dP};
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < CPL; ++k) racc[s][q][k] = 0.f;
    // flush one tap column (0: corners 0/2, 1: corners 1/3) of slot s
    auto flush_col = [&](int s, int col) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int q = col + 2 * r;
        if (rin[s] >> q & 1u) {
          float* row = rrow[s] + (size_t)tap_offset(q, d.w) * twoCv;
#pragma unroll
          for (int k = 0; k < CPL; ++k) {
            int ch = lane + 64 * k;
            if (SCATTER && ch < d.Cv) atomicAdd(row + ch, racc[s][q][k]);
          }
        }
      }
    };
    auto flush = [&](int s) {
      if (rside[s] < 0) return;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (rin[s] >> q & 1u) {
          float* row = rrow[s] + (size_t)tap_offset(q, d.w) * twoCv;
#pragma unroll
          for (int k = 0; k < CPL; ++k) {
            int ch = lane + 64 * k;
            if (SCATTER && ch < d.Cv) atomicAdd(row + ch, racc[s][q][k]);
          }
        }
#pragma unroll
        for (int k = 0; k < CPL; ++k) racc[s][q][k] = 0.f;
      }
    };
    for (int j = 0; j < nvox; ++j) {
      const int cj = rdl(cnt, j);
      if (cj != 1 && cj != 2) continue;
      const size_t vrow = ((size_t)b * V + v0 + j) * d.Cv;
      float dpre[CPL];
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        int ch = lane + 64 * k;
        dpre[k] = 0.f;
        if (ch < d.Cv) {
          float o = vox[vrow + ch];
          dpre[k] = dvox[vrow + ch] * (o > 0.f ? 1.f : 0.1f);
          red[k][3 + (cj - 1)] += dpre[k];
        }
      }
      const int off = (cj == 1) ? 0 : d.Cv;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (s >= cj) break;
        const Tap& tl = s == 0 ? t0 : t1;
        const int cam = rdl(tl.cam, j);
        const int base = rdl(tl.base, j);
        const unsigned in = rdlu(tl.in, j);
        const float zt = rdlf(tl.z, j);
        // run key: (camera, column half) + base pixel; a base one pixel to the right / left keeps
        // the shared tap column in registers (flush only the column that leaves the footprint)
        const int side = (cj == 1 ? 0 : 1) * 8 + cam;
        const int rb = rbase[s], rs = rside[s];
        const unsigned ri = rin[s];
        // a retained column keeps its accumulators only if its in-range bits agree (a base can
        // name two pixels at the row ends: x0 = -1 of row y0 and x0 = w-1 of row y0-1)
        if (side == rs && base == rb + 1 && ((ri >> 1) & 5u) == (in & 5u)) {
          flush_col(s, 0);
#pragma unroll
          for (int k = 0; k < CPL; ++k) {
            racc[s][0][k] = racc[s][1][k];
            racc[s][2][k] = racc[s][3][k];
            racc[s][1][k] = 0.f;
            racc[s][3][k] = 0.f;
          }
        } else if (side == rs && base == rb - 1 && (ri & 5u) == ((in >> 1) & 5u)) {
          flush_col(s, 1);
#pragma unroll
          for (int k = 0; k < CPL; ++k) {
            racc[s][1][k] = racc[s][0][k];
            racc[s][3][k] = racc[s][2][k];
            racc[s][0][k] = 0.f;
            racc[s][2][k] = 0.f;
          }
        } else if (!(side == rs && base == rb && ri == in)) {
          flush(s);
        }
        // the new footprint's in-range bits describe every accumulator (checked above for the
        // retained column; the other column starts at zero)
        rside[s] = side;
        rbase[s] = base;
        rin[s] = in;
        rrow[s] = dP + ((size_t)(b * d.N + cam) * hw + base) * twoCv + off;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float wq = rdlf(tl.w[q], j);
#pragma unroll
          for (int k = 0; k < CPL; ++k) racc[s][q][k] += wq * dpre[k];
        }
        const int zrow = (cj == 1) ? 0 : 1 + d.group[cam];
        const float zf = zt / d.z_scale;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
          // select the row without dynamic register indexing
          float c = dpre[k] * zf;
          red[k][0] += zrow == 0 ? c : 0.f;
          red[k][1] += zrow == 1 ? c : 0.f;
          red[k][2] += zrow == 2 ? c : 0.f;
        }
      }
    }
    flush(0);
    flush(1);
  }
  if (v0 < V) {
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      int ch = lane + 64 * k;
      if (ch < d.Cv)
#pragma unroll
        for (int r = 0; r < 5; ++r) part[r * d.Cv + ch] = red[k][r];
    }
  }
}

__global__ __launch_bounds__(256) void fuse_depth_reduce_k(const float* __restrict__ partial, int n_rows, int n_out,
                                                           float* __restrict__ out) {
  // out[i] = sum_r partial[r, i]: one block per output, fp64 accumulation, fixed order
  __shared__ double lds[4];
  const int i = blockIdx.x;
  double s = 0.0;
  for (int r = threadIdx.x; r < n_rows; r += blockDim.x) s += (double)partial[(size_t)r * n_out + i];
  s = block_sum_all(s, lds);
  if (threadIdx.x == 0) out[i] = (float)s;
}

// ------------------------------------------------------------------------------ fusion plan
// One pass over the voxel grid per step: for every (batch, camera) the compacted list of voxels
// that camera sees, with the tap data every fusion kernel needs.  The geometry depends only on
// K, E and the mask, so the two pose-net calls (forward and backward) share one plan.
struct PlanEntry {
  uint32_t meta;     // voxel index (bits 0-23) | count of valid cameras (24-27) | in-range taps (28-31)
  int32_t base;      // y0 * w + x0
  float fx, fy;      // ix - x0, iy - y0 (exact in fp32; weights are rebuilt bit-identically)
  float z;           // camera-frame depth of the voxel
  float den;         // count + 1e-7 (pose-mode mean denominator, volumetric_fusionnet.py:162)
  int16_t x0, y0;    // tap 0 (may be -1: zeros padding)
  uint32_t pad;
};
static_assert(sizeof(PlanEntry) == 32, "plan entry must stay 32 B");

__device__ __forceinline__ void entry_weights(const PlanEntry& e, float* w) {
  const float ax = 1.f - e.fx, ay = 1.f - e.fy;     // == x1 - ix, y1 - iy exactly
  w[0] = ax * ay;
  w[1] = e.fx * ay;
  w[2] = ax * e.fy;
  w[3] = e.fx * e.fy;
}

template <int NC>
__global__ __launch_bounds__(256) void fusion_plan_k(vfd_voxel_desc d, const float* __restrict__ mlo,
                                                     const float* __restrict__ K, const float* __restrict__ Einv,
                                                     PlanEntry* __restrict__ plan, int* __restrict__ counts) {
  __shared__ int wave_cnt[NC][4];
  __shared__ int block_base[NC];
  const int V = d.X * d.Y * d.Z;
  const int b = blockIdx.y;
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  const int hw = d.h * d.w;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  bool val[NC];
  VoxCam g[NC];
  int cnt = 0;
  if (v < V) {
    const float x = d.axis_x[v % d.X], y = d.axis_y[(v / d.X) % d.Y], z = d.axis_z[v / (d.X * d.Y)];
    VoxProj pj[NC];
    float occ[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) pj[c] = voxel_project(K + (b * NC + c) * 16, Einv + (b * NC + c) * 16, x, y, z, d.h, d.w);
#pragma unroll
    for (int c = 0; c < NC; ++c) occ[c] = mlo[(size_t)(b * NC + c) * hw + voxel_mask_index(pj[c])];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      g[c] = voxel_finish(pj[c], occ[c]);
      val[c] = g[c].valid;
      cnt += val[c] ? 1 : 0;
    }
  } else {
#pragma unroll
    for (int c = 0; c < NC; ++c) val[c] = false;
  }
  // every camera's wave counts, then one thread per camera reserves the block's run of entries:
  // the NC counter atomics are in flight together (two barriers instead of three per camera)
  int before[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const unsigned long long m = __ballot(val[c]);
    before[c] = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wave_cnt[c][wv] = __popcll(m);
  }
  __syncthreads();
  if (threadIdx.x < NC) {
    const int c = threadIdx.x;
    const int tot = wave_cnt[c][0] + wave_cnt[c][1] + wave_cnt[c][2] + wave_cnt[c][3];
    block_base[c] = tot ? atomicAdd(counts + b * NC + c, tot) : 0;
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (val[c]) {
      int off = block_base[c] + before[c];
      for (int k = 0; k < wv; ++k) off += wave_cnt[c][k];
      Bilinear bl = bilinear_taps(g[c].ix, g[c].iy, d.w, d.h);
      PlanEntry e;
      unsigned in = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) in |= (bl.in[k] ? 1u : 0u) << k;
      e.meta = (uint32_t)v | ((uint32_t)cnt << 24) | (in << 28);
      e.base = bl.y0 * d.w + bl.x0;
      e.fx = g[c].ix - floorf(g[c].ix);
      e.fy = g[c].iy - floorf(g[c].iy);
      e.z = g[c].z;
      e.den = (float)cnt + 1e-7f;
      e.x0 = (int16_t)bl.x0;
      e.y0 = (int16_t)bl.y0;
      e.pad = 0;
      plan[((size_t)b * NC + c) * V + off] = e;
    }
  }
}

// ------------------------------------------------------------------------------ K2 forward
// Voxel-major gather (volumetric_fusionnet.py:116-162, pose branch) into the channels-last input
// of reduce_dim's stride-2 conv: out[b][y'][x'][z*(C+1) + c] (NHWC, z-major channels; the conv's
// weight is permuted to match, so the convolution is the reference's).  A workgroup owns
// POSE_TV consecutive voxels: (1) one thread per voxel projects it into every camera (the plan's
// arithmetic), (2) each wave takes two voxels at a time with lanes = channels, reads the four
// bilinear taps of every valid camera from the channels-last feature map (one contiguous C-float
// row per tap), sums the cameras in the reference's order, divides by (count + 1e-7) and stores
// the voxel's C+1 values as one contiguous row at each of its (reflect-padded) positions.  Every
// output element is written exactly once: no memset, no atomics.
constexpr int POSE_TV = 32;
constexpr int POSE_MAXC = 256;      // channels held per lane: ceil(C / 64) <= 4
#ifndef VFD_POSE_VU
#define VFD_POSE_VU 2                 // voxels per wave round: 166 vs 170 (1) / 202 (4) us at config 3
#endif
constexpr int POSE_VU = VFD_POSE_VU;
static_assert(POSE_TV % (4 * POSE_VU) == 0, "K2 forward: voxels per wave round");

// order (nullable): the voxels by azimuth sector around the rig, [8][ocap] (-1 = padding,
// kernels.VoxelSpace.pose_order).  Workgroup k runs sector k % 8 — one XCD (the hardware deals
// workgroups round-robin over the 8 XCDs) — so an XCD gathers the feature rows of the one or two
// cameras facing its sector and each row comes into one L2, instead of every XCD caching every
// camera's map.  Null: voxels in index order, POSE_TV per workgroup.
template <int NC, typename TO>
__global__ __launch_bounds__(256) void fuse_pose_fwd_k(vfd_voxel_desc d, const float* __restrict__ mlo,
                                                       const float* __restrict__ K, const float* __restrict__ Einv,
                                                       const float* __restrict__ feats, const int* __restrict__ order,
                                                       int ocap, TO* __restrict__ out) {
  constexpr int CPL = POSE_MAXC / 64;
  __shared__ int s_base[POSE_TV][NC];
  __shared__ float s_w[POSE_TV][NC][4];
  __shared__ int s_cam[POSE_TV][NC];
  __shared__ unsigned s_in[POSE_TV][NC];
  __shared__ int s_cnt[POSE_TV];
  __shared__ float s_den[POSE_TV];
  __shared__ float s_zf[POSE_TV];
  __shared__ int s_v[POSE_TV];
  const int V = d.X * d.Y * d.Z;
  const int b = blockIdx.y;
  const int hw = d.h * d.w;
  const int C = d.C, C1 = d.C + 1;
  if (threadIdx.x < POSE_TV) {
    const int t = threadIdx.x;
    int v;
    if (order) {
      const int i = (blockIdx.x / 8) * POSE_TV + t;
      v = i < ocap ? order[(blockIdx.x % 8) * ocap + i] : -1;
    } else {
      v = blockIdx.x * POSE_TV + t;
      v = v < V ? v : -1;
    }
    s_v[t] = v;
    int cnt = 0;
    float zsum = 0.f;
    if (v >= 0) {
      const float x = d.axis_x[v % d.X], y = d.axis_y[(v / d.X) % d.Y], z = d.axis_z[v / (d.X * d.Y)];
      VoxProj pj[NC];
      float occ[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) pj[c] = voxel_project(K + (b * NC + c) * 16, Einv + (b * NC + c) * 16, x, y, z, d.h, d.w);
#pragma unroll
      for (int c = 0; c < NC; ++c) occ[c] = mlo[(size_t)(b * NC + c) * hw + voxel_mask_index(pj[c])];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const VoxCam g = voxel_finish(pj[c], occ[c]);
        if (g.valid) {
          const Tap tp = make_tap(c, g, d.h, d.w);
          s_cam[t][cnt] = c;
          s_base[t][cnt] = tp.base;
          s_in[t][cnt] = tp.in;
#pragma unroll
          for (int q = 0; q < 4; ++q) s_w[t][cnt][q] = tp.w[q];
          zsum += g.z / d.z_scale;
          ++cnt;
        }
      }
    }
    s_cnt[t] = cnt;
    s_den[t] = (float)cnt + 1e-7f;
    s_zf[t] = zsum / ((float)cnt + 1e-7f);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float* fb = feats + (size_t)b * NC * hw * C;
  const int P = d.pad_out ? 2 : 0;
  const int Yo = d.Y + P, Xo = d.X + P;
  const size_t pix_stride = (size_t)d.Z * C1;
  TO* ob = out + (size_t)b * Yo * Xo * pix_stride;
  if ((C & 3) == 0) {     // lanes = channel quads: 166 vs 188 us (config 3), 91 vs 101 (config 2)
    // lanes = channel quads: one 16-B load per lane brings a whole tap row (C <= 256), the wave
    // works on POSE_VU voxels at a time (wave-uniform: their camera loops are uniform branches) and
    // issues all their tap rows of one camera round before summing any.  The per-channel arithmetic
    // is the lane-per-channel form's, in the same order (taps, then cameras), so the map is
    // bit-identical to it
    const int cq = min(lane, C / 4 - 1) * 4;        // idle lanes (C < 256) re-read the last quad
    const bool own = lane < C / 4;
    for (int t0 = wv * POSE_VU; t0 < POSE_TV; t0 += 4 * POSE_VU) {
      float4 acc[POSE_VU];
      int cmax = 0;
#pragma unroll
      for (int u = 0; u < POSE_VU; ++u) {
        acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        cmax = max(cmax, s_cnt[t0 + u]);
      }
      for (int j = 0; j < cmax; ++j) {
        float4 f[POSE_VU][4];
#pragma unroll
        for (int u = 0; u < POSE_VU; ++u) {
          const int t = t0 + u;
          const bool act = j < s_cnt[t];
          const float* fc = fb + (size_t)(act ? s_cam[t][j] : 0) * hw * C + cq;
          const int base = act ? s_base[t][j] : 0;
          const unsigned in = act ? s_in[t][j] : 0u;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const bool ok = (in >> q & 1u) != 0u;
            f[u][q] = *reinterpret_cast<const float4*>(fc + (size_t)(ok ? base + tap_offset(q, d.w) : 0) * C);
          }
        }
#pragma unroll
        for (int u = 0; u < POSE_VU; ++u) {
          const int t = t0 + u;
          if (j >= s_cnt[t]) continue;
          const unsigned in = s_in[t][j];
          float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float w = (in >> q & 1u) ? s_w[t][j][q] : 0.f;
            val.x += f[u][q].x * w;
            val.y += f[u][q].y * w;
            val.z += f[u][q].z * w;
            val.w += f[u][q].w * w;
          }
          acc[u].x += val.x;
          acc[u].y += val.y;
          acc[u].z += val.z;
          acc[u].w += val.w;
        }
      }
#pragma unroll
      for (int u = 0; u < POSE_VU; ++u) {
        const int t = t0 + u, v = s_v[t];
        if (v < 0) continue;
        const float den = s_den[t];
        const int xi = v % d.X, yi = (v / d.X) % d.Y, zi = v / (d.X * d.Y);
        int rows[3], cols[3], nr, nc;
        pad_sets(yi, d.Y, d.pad_out, rows, &nr);
        pad_sets(xi, d.X, d.pad_out, cols, &nc);
        const float o[4] = {acc[u].x / den, acc[u].y / den, acc[u].z / den, acc[u].w / den};
        const float zf = s_zf[t];
        for (int a = 0; a < nr; ++a)
          for (int c2 = 0; c2 < nc; ++c2) {
            TO* row = ob + ((size_t)rows[a] * Xo + cols[c2]) * pix_stride + (size_t)zi * C1;
            if (own) {
              // rows start at any element (C + 1 per z): element stores, consecutive across lanes
#pragma unroll
              for (int e = 0; e < 4; ++e) row[cq + e] = (TO)o[e];
            }
            if (lane == 0) row[C] = (TO)zf;
          }
      }
    }
    return;
  }
  // C % 4 != 0: lanes = channels
  for (int t0 = wv * 2; t0 < POSE_TV; t0 += 8) {
    float acc[2][CPL];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int k = 0; k < CPL; ++k) acc[u][k] = 0.f;
    const int cmax = max(s_cnt[t0], s_cnt[t0 + 1]);
    for (int j = 0; j < cmax; ++j) {
      float val[2][CPL];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int t = t0 + u;
#pragma unroll
        for (int k = 0; k < CPL; ++k) val[u][k] = 0.f;
        if (j >= s_cnt[t]) continue;
        const float* fc = fb + (size_t)s_cam[t][j] * hw * C;
        const int base = s_base[t][j];
        const unsigned in = s_in[t][j];
        // out-of-range taps (zeros padding) read pixel 0 with weight 0: branch-free loads
        float f[4][CPL], wq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool ok = (in >> q & 1u) != 0u;
          wq[q] = ok ? s_w[t][j][q] : 0.f;
          const float* row = fc + (size_t)(ok ? base + tap_offset(q, d.w) : 0) * C;
#pragma unroll
          for (int k = 0; k < CPL; ++k) {
            const int ch = lane + 64 * k;
            f[q][k] = row[ch < C ? ch : 0];
          }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int k = 0; k < CPL; ++k) val[u][k] += f[q][k] * wq[q];
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
        if (j < s_cnt[t0 + u]) {
#pragma unroll
          for (int k = 0; k < CPL; ++k) acc[u][k] += val[u][k];
        }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = t0 + u, v = s_v[t];
      if (v < 0) continue;
      const float den = s_den[t];
      const int xi = v % d.X, yi = (v / d.X) % d.Y, zi = v / (d.X * d.Y);
      int rows[3], cols[3], nr, nc;
      pad_sets(yi, d.Y, d.pad_out, rows, &nr);
      pad_sets(xi, d.X, d.pad_out, cols, &nc);
      float o[CPL];
#pragma unroll
      for (int k = 0; k < CPL; ++k) o[k] = acc[u][k] / den;
      const float zf = s_zf[t];
      for (int a = 0; a < nr; ++a)
        for (int c2 = 0; c2 < nc; ++c2) {
          TO* row = ob + ((size_t)rows[a] * Xo + cols[c2]) * pix_stride + (size_t)zi * C1;
#pragma unroll
          for (int k = 0; k < CPL; ++k) {
            const int ch = lane + 64 * k;
            if (ch < C) row[ch] = (TO)o[k];
          }
          if (lane == 0) row[C] = (TO)zf;
        }
    }
  }
}

// ------------------------------------------------------------------------------ K2 backward
// Atomic-free, pixel-major.  LDS float atomics cost ~3 cycles per lane on gfx950 (measured on
// the scatter form of this kernel), so the backward is a gather:
//   plan_index_k     once per step with the plan: per (batch, camera) CSR inverse index
//                    pixel -> [(entry << 2) | tap] of every in-range bilinear tap;
//   fuse_pose_bwd_k  per pixel, lanes = channels: sum (g[voxel] / den) * w_tap over the pixel's
//                    list, g read as contiguous rows of the channels-last d_out (reflect-padding
//                    copies folded back), staged through LDS for coalesced NCHW stores.
constexpr int PIDX_THREADS = 1024;

// K2 backward = the transpose of a bilinear gather: every visible (voxel, camera) pair adds
// w_q * g[voxel] / den to the 4 pixels of its tap footprint.  The pixel map is cut into 4x4
// tiles; each tile owns the bucket of plan entries whose footprint touches it (an entry on a
// tile border is listed by every tile it touches, its weights masked to that tile's taps), so a
// workgroup reads each of its voxel rows from HBM exactly once, accumulates in registers
// (16 pixels x C/64 channels per lane) and writes its tile with plain stores: no atomics, no
// inverse pixel index, no re-reads through L2.
constexpr int PT = 4;              // tile side (pixels)
constexpr int PT2 = PT * PT;

// Reflect-pad fold slot of a border voxel (xi in {1, X-2} or yi in {1, Y-2}; -1 otherwise):
// slot = xi (yi == 1), X + xi (yi == Y-2), 2X + yi (xi == 1), 2X + Y + yi (xi == X-2).
__host__ __device__ __forceinline__ int pose_fold_slot(int xi, int yi, int X, int Y) {
  if (yi == 1) return xi;
  if (yi == Y - 2) return X + xi;
  if (xi == 1) return 2 * X + yi;
  if (xi == X - 2) return 2 * X + Y + yi;
  return -1;
}

struct TileItem {
  uint32_t pz;       // d_out row (padded position * Z + z), or bit 31 | fold-buffer row (slot * Z + z)
  float rden;        // 1 / (count + 1e-7) (volumetric_fusionnet.py:162)
  float w[4];        // ATen bilinear weights of taps (x0,y0) (x0+1,y0) (x0,y0+1) (x0+1,y0+1); 0 outside the tile
  int32_t lxy;       // tap 0 relative to the tile origin: (ly + 1) * 8 + (lx + 1), lx, ly in [-1, PT-1]
  uint32_t vc;       // voxel index (bits 0-23) | its count of valid cameras (24-27): K1's gather backward
};
static_assert(sizeof(TileItem) == 32, "tile item must stay 32 B");

// Inside a tile, items are bucketed by their 2x2 footprint position (lx, ly) in [-1, PT-1]^2
// (PSUB = 25 sub-keys), so the backward sums runs of equal footprints in fixed registers and
// touches the pixel-indexed accumulators once per run.
constexpr int PSUB = (PT + 1) * (PT + 1);
__host__ __device__ __forceinline__ int sub_key(int lx, int ly) { return (ly + 1) * (PT + 1) + lx + 1; }

__device__ __forceinline__ int tiles_x(const vfd_voxel_desc& d) { return (d.w + PT - 1) / PT; }
__device__ __forceinline__ int tiles_y(const vfd_voxel_desc& d) { return (d.h + PT - 1) / PT; }

// Tiles touched by an entry's in-range taps: bit (ty - ty0) * 2 + (tx - tx0) over the 2x2 tile
// block starting at (tx0, ty0) = tile of tap 0 (taps out of the map never count).
__device__ __forceinline__ unsigned entry_tiles(const vfd_voxel_desc& d, const PlanEntry& e, int* tx0, int* ty0) {
  const unsigned in = e.meta >> 28;
  const int x0 = e.x0, y0 = e.y0;
  // tap 0 may sit at x0 = -1 / y0 = -1 (left/top zeros padding): floor division
  *tx0 = x0 >= 0 ? x0 / PT : -1;
  *ty0 = y0 >= 0 ? y0 / PT : -1;
  unsigned m = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (in >> q & 1u) {
      const int x = x0 + (q & 1), y = y0 + (q >> 1);
      m |= 1u << ((y / PT - *ty0) * 2 + (x / PT - *tx0));
    }
  return m;
}

// Tile counters see ~100 adders each; a workgroup first histograms its 256 entries in LDS and
// then adds one count per touched tile (entries of one workgroup are neighbouring voxels, so
// they touch a handful of tiles).
__global__ __launch_bounds__(256) void plan_count_k(vfd_voxel_desc d, const PlanEntry* __restrict__ plan,
                                                    const int* __restrict__ counts, int* __restrict__ tile_cnt) {
  extern __shared__ int hist[];          // [nt * PSUB]
  const int bc = blockIdx.y;
  const int V = d.X * d.Y * d.Z, ntx = tiles_x(d), nt = ntx * tiles_y(d), nk = nt * PSUB;
  const int n = counts[bc];
  if ((int)(blockIdx.x * blockDim.x) >= n) return;     // whole workgroup beyond the list
  for (int i = threadIdx.x; i < nk; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const PlanEntry e = plan[(size_t)bc * V + i];
    int tx0, ty0;
    const unsigned m = entry_tiles(d, e, &tx0, &ty0);
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (m >> t & 1u) {
        const int tx = tx0 + (t & 1), ty = ty0 + (t >> 1);
        atomicAdd(hist + (ty * ntx + tx) * PSUB + sub_key(e.x0 - tx * PT, e.y0 - ty * PT), 1);
      }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < nk; t += blockDim.x)
    if (hist[t]) atomicAdd(tile_cnt + (size_t)bc * nk + t, hist[t]);
}

__global__ __launch_bounds__(PIDX_THREADS) void plan_scan_k(vfd_voxel_desc d, int* __restrict__ tile_cnt,
                                                            int* __restrict__ tile_ptr) {
  // exclusive scan of the bucket counts: wave prefix sums by lane shuffles + one cross-wave step
  constexpr int NW = PIDX_THREADS / 64;
  __shared__ int wsum[NW];
  const int nt = tiles_x(d) * tiles_y(d) * PSUB;     // (tile, sub-key) buckets
  const int bc = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  int* cnt = tile_cnt + (size_t)bc * nt;
  const int chunk = (nt + PIDX_THREADS - 1) / PIDX_THREADS;
  const int c0 = min(nt, t * chunk), c1 = min(nt, c0 + chunk);
  int local = 0;
  for (int i = c0; i < c1; ++i) local += cnt[i];
  int v = local;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int n = __shfl_up(v, off, 64);
    if (lane >= off) v += n;
  }
  if (lane == 63) wsum[wv] = v;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const int sk = wsum[k];
    base += k < wv ? sk : 0;
    tot += sk;
  }
  int run = base + v - local;
  int* tp = tile_ptr + (size_t)bc * (nt + 1);
  for (int i = c0; i < c1; ++i) {
    const int c = cnt[i];
    tp[i] = run;
    cnt[i] = run;                 // becomes the fill cursor
    run += c;
  }
  if (t == PIDX_THREADS - 1) tp[nt] = tot;
}

__global__ __launch_bounds__(256) void plan_fill_k(vfd_voxel_desc d, const PlanEntry* __restrict__ plan,
                                                   const int* __restrict__ counts, int* __restrict__ cursor,
                                                   TileItem* __restrict__ items) {
  extern __shared__ int lds[];           // [nk] local counts -> slot bases | [nk] local cursors
  const int bc = blockIdx.y;
  const int V = d.X * d.Y * d.Z, ntx = tiles_x(d), nt = ntx * tiles_y(d), nk = nt * PSUB;
  const int n = counts[bc];
  if ((int)(blockIdx.x * blockDim.x) >= n) return;
  int* lbase = lds;
  int* lcur = lds + nk;
  for (int t = threadIdx.x; t < nk; t += blockDim.x) lbase[t] = lcur[t] = 0;
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < n;
  PlanEntry e;
  unsigned m = 0;
  int tx0 = 0, ty0 = 0;
  if (act) {
    e = plan[(size_t)bc * V + i];
    m = entry_tiles(d, e, &tx0, &ty0);
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (m >> t & 1u) {
        const int tx = tx0 + (t & 1), ty = ty0 + (t >> 1);
        atomicAdd(lbase + (ty * ntx + tx) * PSUB + sub_key(e.x0 - tx * PT, e.y0 - ty * PT), 1);
      }
  }
  __syncthreads();
  int* cur = cursor + (size_t)bc * nk;
  for (int t = threadIdx.x; t < nk; t += blockDim.x)
    if (lbase[t]) lbase[t] = atomicAdd(cur + t, lbase[t]);
  __syncthreads();
  if (!act) return;
  const unsigned in = e.meta >> 28;
  const int v = (int)(e.meta & 0xFFFFFF);
  const int xi = v % d.X, yi = (v / d.X) % d.Y, zi = v / (d.X * d.Y);
  const int P1 = d.pad_out ? 1 : 0;
  const bool fold = d.pad_out && (xi == 1 || xi == d.X - 2 || yi == 1 || yi == d.Y - 2);
  TileItem it;
  it.pz = fold ? (1u << 31) | (uint32_t)(pose_fold_slot(xi, yi, d.X, d.Y) * d.Z + zi)
               : (uint32_t)(((yi + P1) * (d.X + 2 * P1) + xi + P1) * d.Z + zi);
  it.rden = 1.f / e.den;
  it.vc = e.meta & 0x0FFFFFFFu;
  float w[4];
  entry_weights(e, w);
  const int x0 = e.x0, y0 = e.y0;
  TileItem* ib = items + (size_t)bc * 4 * V;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (!(m >> t & 1u)) continue;
    const int tx = tx0 + (t & 1), ty = ty0 + (t >> 1), tile = ty * ntx + tx;
    const int lx = x0 - tx * PT, ly = y0 - ty * PT;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int px = lx + (q & 1), py = ly + (q >> 1);
      const bool mine = (in >> q & 1u) && px >= 0 && px < PT && py >= 0 && py < PT;
      it.w[q] = mine ? w[q] : 0.f;
    }
    it.lxy = (ly + 1) * 8 + (lx + 1);
    const int key = tile * PSUB + sub_key(lx, ly);
    ib[lbase[key] + atomicAdd(lcur + key, 1)] = it;
  }
}

// Deterministic mode: the fill above orders a bucket's items by atomic arrival.  plan_order_k
// ranks every item within its (tile, sub-key) bucket by voxel index (unique in a bucket: an entry
// lists a tile once) into `tmp`; plan_copy_k moves them back.  Buckets are short (tens of
// items), so the rank is a plain count over the bucket.
__global__ __launch_bounds__(256) void plan_order_k(vfd_voxel_desc d, const int* __restrict__ row_ptr,
                                                    const TileItem* __restrict__ items, TileItem* __restrict__ tmp) {
  const int bc = blockIdx.y;
  const int V = d.X * d.Y * d.Z, nk = tiles_x(d) * tiles_y(d) * PSUB;
  const int* tp = row_ptr + (size_t)bc * (nk + 1);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tp[nk]) return;
  int lo = 0, hi = nk;                              // last bucket k with tp[k] <= i
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (tp[mid] <= i) lo = mid; else hi = mid;
  }
  const TileItem* ib = items + (size_t)bc * 4 * V;
  const TileItem it = ib[i];
  const uint32_t key = it.vc & 0xFFFFFFu;
  int r = 0;
  for (int j = tp[lo]; j < tp[lo + 1]; ++j) r += (ib[j].vc & 0xFFFFFFu) < key ? 1 : 0;
  tmp[(size_t)bc * 4 * V + tp[lo] + r] = it;
}

__global__ __launch_bounds__(256) void plan_copy_k(vfd_voxel_desc d, const int* __restrict__ row_ptr,
                                                   const TileItem* __restrict__ tmp, TileItem* __restrict__ items) {
  const int bc = blockIdx.y;
  const int V = d.X * d.Y * d.Z, nk = tiles_x(d) * tiles_y(d) * PSUB;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= row_ptr[(size_t)bc * (nk + 1) + nk]) return;
  items[(size_t)bc * 4 * V + i] = tmp[(size_t)bc * 4 * V + i];
}

// Load balance of the backward: tiles at the horizon collect ~4x the mean item count.  A tile
// with more than PBW_SPLIT items is split into S <= PBW_MAXS item ranges ("parts", ~PBW_PART
// items each); each part writes its partial tile into a pool slot and a second launch sums the
// S slots in part order into d_feats (deterministic: no float atomics; an in-launch hand-off to
// the last part measured slower: its serial cross-XCD slot reads stretch the tail).  Split
// tiles are queued first.
//   tasks[i]  = {bc * nt + tile, lo, hi, meta}: items [lo, hi) of the (bc) item block;
//               meta = -1 for a whole tile, else the part's pool slot
//   combos[k] = {bc * nt + tile, first slot, S, 0} for the k-th split tile
//   ctrl      = {task count, split-tile count}
// When the pool runs out, the remaining heavy tiles run whole (correct, just slower).
#ifndef VFD_PBW_SPLIT
#define VFD_PBW_SPLIT 128
#endif
#ifndef VFD_PBW_PART
#define VFD_PBW_PART 104
#endif
constexpr int PBW_SPLIT = VFD_PBW_SPLIT;
constexpr int PBW_PART = VFD_PBW_PART;
constexpr int PBW_MAXS = 8;
constexpr int PBW_POOL = 8192;         // part slots of PT2 x POSE_MAXC floats (128 MB)

__global__ __launch_bounds__(1024) void plan_task_k(vfd_voxel_desc d, const int* __restrict__ tile_ptr,
                                                    int4* __restrict__ tasks, int4* __restrict__ combos,
                                                    int* __restrict__ ctrl) {
  // One workgroup: four exclusive scans over the (batch, camera, tile) list.  Scans are wave
  // prefix sums by lane shuffles plus one cross-wave step (two barriers each), and a thread's
  // tile ranges are read once into registers (the first version re-read them per pass and ran
  // 1024-wide LDS scans: ~20 us of barriers and round trips for a few KB).
  constexpr int TASK_T = 1024, TASK_W = TASK_T / 64, TASK_CACHE = 8;
  __shared__ int wsum[TASK_W];
  const int nt = tiles_x(d) * tiles_y(d);
  const int M = d.B * d.N * nt;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int chunk = (M + TASK_T - 1) / TASK_T;
  const int c0 = min(M, t * chunk), c1 = min(M, c0 + chunk);
  auto range_ld = [&](int i, int& lo, int& hi) {
    const int bc = i / nt, tile = i % nt;
    const int* tp = tile_ptr + (size_t)bc * (nt * PSUB + 1);
    lo = tp[tile * PSUB];
    hi = tp[(tile + 1) * PSUB];
  };
  int clo[TASK_CACHE], chi[TASK_CACHE];
#pragma unroll
  for (int j = 0; j < TASK_CACHE; ++j)
    if (c0 + j < c1) range_ld(c0 + j, clo[j], chi[j]);
  auto range = [&](int i, int& lo, int& hi) {
    const int j = i - c0;
    if (j < TASK_CACHE) {
#pragma unroll
      for (int q = 0; q < TASK_CACHE; ++q)
        if (q == j) { lo = clo[q]; hi = chi[q]; }
    } else {
      range_ld(i, lo, hi);
    }
  };
  auto want = [](int n) { return n > PBW_SPLIT ? min(PBW_MAXS, (n + PBW_PART - 1) / PBW_PART) : 0; };
  int total = 0;
  auto scan = [&](int local) {                     // exclusive prefix over threads; sum -> `total`
    int v = local;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int n = __shfl_up(v, off, 64);
      if (lane >= off) v += n;
    }
    __syncthreads();                               // the previous scan's wsum reads are done
    if (lane == 63) wsum[wv] = v;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < TASK_W; ++k) {
      const int sk = wsum[k];
      base += k < wv ? sk : 0;
      tot += sk;
    }
    total = tot;
    return base + v - local;
  };
  int lo, hi;
  // pass 0: pool slots wanted
  int local = 0;
  for (int i = c0; i < c1; ++i) { range(i, lo, hi); local += want(hi - lo); }
  const int slot0 = scan(local);
  auto fits = [](int s, int sl) { return s > 0 && sl + s <= PBW_POOL; };
  // pass 1: split tiles (their slots fit the pool): parts and combine entries
  int nsplit = 0, nwhole = 0;
  local = 0;
  for (int i = c0, sl = slot0; i < c1; ++i) {
    range(i, lo, hi);
    const int s = want(hi - lo);
    if (fits(s, sl)) { local += s; ++nsplit; } else { ++nwhole; }
    sl += s;
  }
  int run = scan(local);
  const int n_parts = total;
  int crun = scan(nsplit);
  const int n_combo = total;
  int wrun = scan(nwhole);                         // pass 2 (whole tiles) goes after the parts
  const int n_whole = total;
  wrun += n_parts;
  for (int i = c0, sl = slot0; i < c1; ++i) {
    range(i, lo, hi);
    const int n = hi - lo, s = want(n);
    if (fits(s, sl)) {
      for (int p = 0; p < s; ++p)
        tasks[run++] = make_int4(i, lo + (int)((long long)n * p / s), lo + (int)((long long)n * (p + 1) / s), sl + p);
      combos[crun++] = make_int4(i, sl, s, 0);
    } else {
      tasks[wrun++] = make_int4(i, lo, hi, -1);
    }
    sl += s;
  }
  if (t == 0) {
    ctrl[0] = n_parts + n_whole;
    ctrl[1] = n_combo;
  }
}

#ifndef VFD_PBW_U
#define VFD_PBW_U 8
#endif
constexpr int PBW_U = VFD_PBW_U;       // voxel rows (1 KB each) in flight per wave

// Reflect-pad fold of the pose output's gradient: a voxel with xi in {1, X-2} or yi in {1, Y-2}
// has copies in the padded map; their sum goes to a compact buffer (row = (b * nslot + slot) * Z
// + z, C + 1 floats), so the backward's row reads carry no data-dependent extra loads.
// grid = B * nslot * POSE_FOLD_SPLIT: each slot's Z * (C + 1) floats are split over
// POSE_FOLD_SPLIT workgroups (a slot per workgroup leaves 400 workgroups on 256 CUs, latency-bound)
constexpr int POSE_FOLD_SPLIT = 4;
template <typename TG>
__global__ __launch_bounds__(256) void pose_fold_k(vfd_voxel_desc d, const TG* __restrict__ dout,
                                                   float* __restrict__ fb, int aligned16) {
  const int nslot = 2 * (d.X + d.Y);
  const int part = blockIdx.x % POSE_FOLD_SPLIT, sb = blockIdx.x / POSE_FOLD_SPLIT;
  const int slot = sb % nslot, b = sb / nslot;
  int xi, yi;
  if (slot < d.X) { xi = slot; yi = 1; }
  else if (slot < 2 * d.X) { xi = slot - d.X; yi = d.Y - 2; }
  else if (slot < 2 * d.X + d.Y) { xi = 1; yi = slot - 2 * d.X; }
  else { xi = d.X - 2; yi = slot - 2 * d.X - d.Y; }
  if (pose_fold_slot(xi, yi, d.X, d.Y) != slot) return;     // owned by an earlier slot
  // a padded position's Z rows are contiguous: sum the (up to 4) copies' Z * (C + 1) floats
  const int n = d.Z * (d.C + 1), Xo = d.X + 2;
  const TG* gb = dout + (size_t)b * (d.Y + 2) * Xo * n;
  const int ex = xi == 1 ? 0 : (xi == d.X - 2 ? d.X + 1 : -1);   // x-mirror column (padded)
  const int ey = yi == 1 ? 0 : (yi == d.Y - 2 ? d.Y + 1 : -1);
  const TG* p0 = gb + ((size_t)(yi + 1) * Xo + xi + 1) * n;
  const TG* p1 = gb + ((size_t)(yi + 1) * Xo + max(ex, 0)) * n;
  const TG* p2 = gb + ((size_t)max(ey, 0) * Xo + xi + 1) * n;
  const TG* p3 = gb + ((size_t)max(ey, 0) * Xo + max(ex, 0)) * n;
  const float f1 = ex >= 0 ? 1.f : 0.f, f2 = ey >= 0 ? 1.f : 0.f, f3 = f1 * f2;
  float* dst = fb + ((size_t)b * nslot + slot) * n;
  // ((primary + x-copy) + y-copy) + xy-copy, absent copies weighted 0 (loads stay in range)
  if (sizeof(TG) == 4 && (n & 3) == 0 && aligned16) {   // fp32 rows start 16-B aligned: float4 lanes
    const int n4 = n >> 2, c4 = (n4 + POSE_FOLD_SPLIT - 1) / POSE_FOLD_SPLIT;
    const int e4 = min(n4, (part + 1) * c4);
    const float4 *q0 = reinterpret_cast<const float4*>(p0), *q1 = reinterpret_cast<const float4*>(p1);
    const float4 *q2 = reinterpret_cast<const float4*>(p2), *q3 = reinterpret_cast<const float4*>(p3);
    for (int i = part * c4 + threadIdx.x; i < e4; i += blockDim.x) {
      const float4 a = q0[i], bx = q1[i], by = q2[i], bxy = q3[i];
      float4 r;
      r.x = ((a.x + f1 * bx.x) + f2 * by.x) + f3 * bxy.x;
      r.y = ((a.y + f1 * bx.y) + f2 * by.y) + f3 * bxy.y;
      r.z = ((a.z + f1 * bx.z) + f2 * by.z) + f3 * bxy.z;
      r.w = ((a.w + f1 * bx.w) + f2 * by.w) + f3 * bxy.w;
      reinterpret_cast<float4*>(dst)[i] = r;
    }
    return;
  }
  const int cn = (n + POSE_FOLD_SPLIT - 1) / POSE_FOLD_SPLIT, e = min(n, (part + 1) * cn);
  for (int i = part * cn + threadIdx.x; i < e; i += blockDim.x) {
    float s = ld1(p0 + i);
    s += f1 * ld1(p1 + i);
    s += f2 * ld1(p2 + i);
    s += f3 * ld1(p3 + i);
    dst[i] = s;
  }
}

#ifdef VFD_PBW_TRACE
// diagnostic build only: per wave task {start, end, items | split << 24, cu | group << 32} (100 MHz clock)
__device__ unsigned long long g_pbw_trace[16384 * 4];
extern "C" int vfd_pbw_trace_read(void* dst, size_t bytes) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_pbw_trace), bytes, 0, hipMemcpyDeviceToHost);
}
#endif

// One single-wave workgroup per task (a tile, or a part of a split tile); each lane owns four
// consecutive channels, so one 16-B-per-lane load brings a whole gradient row (C <= 256
// channels, 1 KiB) per wave-instruction.  The wave walks the task's items in batches of PBW_U
// (records fetched lane-parallel four batches ahead and broadcast by readlane, rows loaded one
// batch ahead), sums each footprint run in registers and flushes it into its LDS tile
// [PT2 + 1][256] (row PT2 takes taps outside the tile).  Rows start at any 4-B offset (C + 1
// floats per row): the 16-B loads run unaligned, which gfx9's unaligned access mode allows.
template <typename TG>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3))) void fuse_pose_bwd_k(vfd_voxel_desc d, const int4* __restrict__ tasks,
                                                      const int* __restrict__ ctrl, const TileItem* __restrict__ items,
                                                      const TG* __restrict__ dout, const float* __restrict__ fbuf,
                                                      float* __restrict__ pool, float* __restrict__ dfeats) {
  constexpr int U = PBW_U;
  constexpr int PR = PT2 + 1;
  __shared__ float4 acc_l[PR * 64];
  const int lane = threadIdx.x;
  const int wt = xcd_task(ctrl[0]);              // neighbouring tiles on one XCD (shared rows in its L2)
  if (wt < 0) return;
#ifdef VFD_PBW_TRACE
  const unsigned long long t_start = wall_clock64();
#endif
  const int C = d.C, C1 = d.C + 1;
  const int4 rec = tasks[wt];
  const int bct = rec.x, lo = rec.y, hi = rec.z, meta = rec.w;
  const int nt = tiles_x(d) * tiles_y(d), ntx = tiles_x(d);
  const int bc = bct / nt, b = bc / d.N, tile = bct % nt;
  const int V = d.X * d.Y * d.Z, hw = d.h * d.w;
  const int P = d.pad_out ? 2 : 0;
  const TG* gb = dout + (size_t)b * (d.Y + P) * (d.X + P) * d.Z * C1;
  const float* fb = fbuf + (size_t)b * 2 * (d.X + d.Y) * d.Z * C1;
  const TileItem* ib = items + (size_t)bc * 4 * V;
  const int cq = min(lane, C / 4 - 1) * 4;         // this lane's first channel (idle lanes re-read)
  float4* wacc = acc_l + lane;
#pragma unroll
  for (int p = 0; p < PT2; ++p) wacc[64 * p] = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 tq[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) tq[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  int cur = -1;
  auto flush = [&]() {
    if (cur < 0) return;
    const int lx = (cur & 7) - 1, ly = (cur >> 3) - 1;
    int o[4];
    float4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int px = lx + (q & 1), py = ly + (q >> 1);
      o[q] = 64 * ((px >= 0 && px < PT && py >= 0 && py < PT) ? py * PT + px : PT2);
      v[q] = wacc[o[q]];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      wacc[o[q]] = make_float4(v[q].x + tq[q].x, v[q].y + tq[q].y, v[q].z + tq[q].z, v[q].w + tq[q].w);
      tq[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  // lane-parallel record fetch of a group of 3 batches: lane i < 3U holds item jb + i; tail
  // slots re-read the last item and get 1/den = 0 when consumed (they add nothing and keep its
  // footprint: no flush).  A fetched record is never touched before its use (any VALU op on it
  // would wait for it).
  constexpr int GI = 3 * U;                        // items per record group
  auto fetch = [&](int jb) { return ib[min(jb + (lane < GI ? lane : 0), hi - 1)]; };
  // the item's gradient row: its own padded position, or the folded sum of its reflect copies
  // (bit 31): a wave-uniform pointer select, so every row load is unconditional
  // (buffer loads: the row offset is a scalar soffset and the lane's channel offset a constant
  // voffset, so an item costs no VGPR address arithmetic)
  const __amdgpu_buffer_rsrc_t rs_g = __builtin_amdgcn_make_buffer_rsrc(
      (void*)gb, 0, (int)((size_t)(d.Y + P) * (d.X + P) * d.Z * C1 * sizeof(TG)), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_f = __builtin_amdgcn_make_buffer_rsrc(
      (void*)fb, 0, (int)((size_t)2 * (d.X + d.Y) * d.Z * C1 * sizeof(float)), 0x00020000);
  const int voff = cq * (int)sizeof(float);
  auto issue = [&](const TileItem& m, int k, float4 (&gr)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)m.pz, k * U + u);
      if constexpr (sizeof(TG) == 4) {
        const int soff = (int)((r & 0x7FFFFFFFu) * (uint32_t)C1 * (uint32_t)sizeof(float));
        const auto v = __builtin_amdgcn_raw_buffer_load_b128((r >> 31) ? rs_f : rs_g, voff, soff, 0);
        gr[u] = make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
      } else if (r >> 31) {                      // folded border row: fp32 sums (wave-uniform branch)
        const int soff = (int)((r & 0x7FFFFFFFu) * (uint32_t)C1 * (uint32_t)sizeof(float));
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs_f, voff, soff, 0);
        gr[u] = make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
      } else {                                   // bf16 gradient row: 4 channels in 8 B
        const int soff = (int)(r * (uint32_t)C1 * 2u);
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs_g, cq * 2, soff, 0);
        gr[u] = make_float4(__uint_as_float((uint32_t)v[0] << 16), __uint_as_float((uint32_t)v[0] & 0xFFFF0000u),
                            __uint_as_float((uint32_t)v[1] << 16), __uint_as_float((uint32_t)v[1] & 0xFFFF0000u));
      }
    }
  };
  auto consume = [&](int jb, const TileItem& m, int k, const float4 (&gr)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int lxy = __builtin_amdgcn_readlane(m.lxy, k * U + u);
      if (lxy != cur) {
        flush();
        cur = lxy;
      }
      // d(mean) = g / den (as g * (1/den)), then grid_sample's backward adds d(mean) * w
      const float rden = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m.rden), k * U + u));
      const float r = jb + u < hi ? rden : 0.f;
      const float4 gd = make_float4(gr[u].x * r, gr[u].y * r, gr[u].z * r, gr[u].w * r);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m.w[q]), k * U + u));
        tq[q].x = __builtin_fmaf(gd.x, w, tq[q].x);
        tq[q].y = __builtin_fmaf(gd.y, w, tq[q].y);
        tq[q].z = __builtin_fmaf(gd.z, w, tq[q].z);
        tq[q].w = __builtin_fmaf(gd.w, w, tq[q].w);
      }
    }
  };
  // rows: a 3-slot ring, two batches in flight beyond the one being summed; records: the
  // current and the next group, alternating between two registers (no copies)
  float4 s0[U], s1[U], s2[U];
  auto group = [&](int jg, const TileItem& Rc, const TileItem& Rn) {
    issue(Rc, 2, s2);
    consume(jg, Rc, 0, s0);
    issue(Rn, 0, s0);
    consume(jg + U, Rc, 1, s1);
    issue(Rn, 1, s1);
    consume(jg + 2 * U, Rc, 2, s2);
  };
  TileItem R0 = fetch(lo), R1 = fetch(lo + GI);
  issue(R0, 0, s0);
  issue(R0, 1, s1);
  for (int j = lo;; j += 2 * GI) {
    group(j, R0, R1);
    if (j + GI >= hi) break;
    R0 = fetch(j + 2 * GI);
    group(j + GI, R1, R0);
    if (j + 2 * GI >= hi) break;
    R1 = fetch(j + 3 * GI);
  }
  flush();
#ifdef VFD_PBW_TRACE
  if (lane == 0 && wt < 16384) {
    unsigned long long* r = g_pbw_trace + 4 * wt;
    r[0] = t_start;
    r[1] = wall_clock64();
    r[2] = (unsigned long long)(hi - lo) | ((unsigned long long)(meta >= 0) << 24);
    r[3] = (unsigned long long)__smid();
  }
#endif
  if (meta >= 0) {                                 // a split tile's part: its pool slot
    float4* ps = reinterpret_cast<float4*>(pool + (size_t)meta * PT2 * POSE_MAXC) + lane;
    if (4 * lane < C) {
#pragma unroll
      for (int p = 0; p < PT2; ++p) ps[p * (POSE_MAXC / 4)] = wacc[64 * p];
    }
    return;
  }
  // NCHW: each lane writes 4 x-consecutive pixels of one channel per store (ch = lane + 64 k)
  const float* tl = reinterpret_cast<const float*>(acc_l);      // [PR][256] floats
  const int tx = tile % ntx, ty = tile / ntx;
  const int x0 = tx * PT;
  float* db = dfeats + (size_t)bc * C * hw;
  const bool vec = (d.w % 4) == 0 && x0 + PT <= d.w;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int ch = lane + 64 * k;
    if (ch >= C) break;
#pragma unroll
    for (int py = 0; py < PT; ++py) {
      const int y = ty * PT + py;
      if (y >= d.h) break;
      float v[PT];
#pragma unroll
      for (int px = 0; px < PT; ++px) v[px] = tl[(py * PT + px) * 256 + ch];
      float* dst = db + (size_t)ch * hw + (size_t)y * d.w + x0;
      if (vec) {
        *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int px = 0; px < PT; ++px)
          if (x0 + px < d.w) dst[px] = v[px];
      }
    }
  }
}

// Split tiles: the S part slots summed in part order.  A workgroup takes split tiles in turn;
// thread = (tile row, channel): all PT rows at once (one round of S x PT slot loads per thread,
// the rows in flight together instead of one after another: 19.3 -> 17.9 us per call at config 2
// under rocprofv3 — the row order was not what held it; it reads S partial tiles of 16 KB per split tile),
// each channel's 4 pixels of a row written as one 16-B store.
constexpr int PCB_THREADS = PT * POSE_MAXC;
__global__ __launch_bounds__(PCB_THREADS) void pose_combine_k(vfd_voxel_desc d, const int4* __restrict__ combos,
                                                              const int* __restrict__ ctrl, const float* __restrict__ pool,
                                                              float* __restrict__ dfeats) {
  const int nt = tiles_x(d) * tiles_y(d), ntx = tiles_x(d);
  const int hw = d.h * d.w;
  const int ch = threadIdx.x % POSE_MAXC, py = threadIdx.x / POSE_MAXC;
  const int ncombo = ctrl[1];
  const bool vec = (d.w % 4) == 0;
  for (int k = blockIdx.x; k < ncombo; k += gridDim.x) {
    const int4 cb = combos[k];
    const int bc = cb.x / nt, tile = cb.x % nt;
    const int x0 = (tile % ntx) * PT, y0 = (tile / ntx) * PT;
    if (ch >= d.C || y0 + py >= d.h) continue;
    const float* p0 = pool + (size_t)cb.y * PT2 * POSE_MAXC + ch;
    float* db = dfeats + ((size_t)bc * d.C + ch) * hw;
    // every slot load unconditional (absent parts re-read the last slot and add +0)
    float v[PBW_MAXS][PT];
#pragma unroll
    for (int s = 0; s < PBW_MAXS; ++s)
#pragma unroll
      for (int px = 0; px < PT; ++px)
        v[s][px] = p0[((size_t)min(s, cb.z - 1) * PT2 + py * PT + px) * POSE_MAXC];
    float a[PT];
#pragma unroll
    for (int px = 0; px < PT; ++px) {
      a[px] = v[0][px];
#pragma unroll
      for (int s = 1; s < PBW_MAXS; ++s) a[px] += (s < cb.z ? 1.f : 0.f) * v[s][px];   // part order
    }
    float* dst = db + (size_t)(y0 + py) * d.w + x0;
    if (vec && x0 + PT <= d.w) {
      *reinterpret_cast<float4*>(dst) = make_float4(a[0], a[1], a[2], a[3]);
    } else {
#pragma unroll
      for (int px = 0; px < PT; ++px)
        if (x0 + px < d.w) dst[px] = a[px];
    }
  }
}

// ------------------------------------------------------------------------------ K1 backward (gather)
// The K1 backward's d P as a gather over the fusion plan's tile buckets (the K2 backward's index:
// the geometry is the same): per (batch, camera, 4x4 pixel tile) task, lanes = the Cv = 64 voxel
// channels; every item (a visible (voxel, camera) pair touching the tile) with a camera count of 1
// or 2 adds w_tap * d pre-activation to its footprint's pixels in the non-overlap (count 1) or
// overlap (count 2) half of the tile's d P rows, runs of equal footprints summed in registers.
// No atomics; d P is written once with plain stores (split tiles through the pool + combine in
// part order), so the result depends only on the item order of each bucket.
constexpr int K1G_CV = 64;

__global__ __launch_bounds__(64) void fuse_depth_bwd_gather_k(vfd_voxel_desc d, const int4* __restrict__ tasks,
                                                              const int* __restrict__ ctrl,
                                                              const TileItem* __restrict__ items,
                                                              const float* __restrict__ dvox,
                                                              const float* __restrict__ vox,
                                                              float* __restrict__ pool, float* __restrict__ dP) {
  constexpr int PR = PT2 + 1, ROW = 2 * K1G_CV;
  constexpr int U = 8;
  __shared__ float acc_l[PR * ROW];
  const int lane = threadIdx.x;
  const int wt = xcd_task(ctrl[0]);
  if (wt < 0) return;
  const int4 rec = tasks[wt];
  const int bct = rec.x, lo = rec.y, hi = rec.z, meta = rec.w;
  const int nt = tiles_x(d) * tiles_y(d), ntx = tiles_x(d);
  const int bc = bct / nt, b = bc / d.N, tile = bct % nt;
  const int V = d.X * d.Y * d.Z, hw = d.h * d.w;
  const TileItem* ib = items + (size_t)bc * 4 * V;
  const float* gv = dvox + (size_t)b * V * K1G_CV + lane;
  const float* ov = vox + (size_t)b * V * K1G_CV + lane;
#pragma unroll
  for (int p = 0; p < PR; ++p) {
    acc_l[p * ROW + lane] = 0.f;
    acc_l[p * ROW + K1G_CV + lane] = 0.f;
  }
  float tq[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int q = 0; q < 4; ++q) tq[h][q] = 0.f;
  int cur = -1;
  auto flush = [&]() {
    if (cur < 0) return;
    const int lx = (cur & 7) - 1, ly = (cur >> 3) - 1;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int px = lx + (q & 1), py = ly + (q >> 1);
      float* a = acc_l + ((px >= 0 && px < PT && py >= 0 && py < PT) ? py * PT + px : PT2) * ROW + lane;
      a[0] += tq[0][q];
      a[K1G_CV] += tq[1][q];
      tq[0][q] = tq[1][q] = 0.f;
    }
  };
  // batches of U items, software-pipelined: records fetched lane-parallel two batches ahead
  // (lane u < U holds item j + u), the next batch's rows loaded while the current one is summed
  auto fetch = [&](int j) { return ib[min(j + (lane < U ? lane : 0), hi - 1)]; };
  auto load = [&](const TileItem& m, float (&g)[U], float (&o)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t vc = (uint32_t)__builtin_amdgcn_readlane((int)m.vc, u);
      const size_t row = (size_t)(vc & 0xFFFFFFu) * K1G_CV;
      g[u] = gv[row];
      o[u] = ov[row];
    }
  };
  auto consume = [&](int j, const TileItem& m, const float (&g)[U], const float (&o)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int lxy = __builtin_amdgcn_readlane(m.lxy, u);
      const uint32_t vc = (uint32_t)__builtin_amdgcn_readlane((int)m.vc, u);
      const int cnt = (int)(vc >> 24);
      const bool live = j + u < hi && (cnt == 1 || cnt == 2);
      if (lxy != cur) {
        flush();
        cur = lxy;
      }
      const float dpre = live ? g[u] * (o[u] > 0.f ? 1.f : 0.1f) : 0.f;
      const float d0 = cnt == 2 ? 0.f : dpre, d1 = cnt == 2 ? dpre : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m.w[q]), u));
        tq[0][q] += w * d0;
        tq[1][q] += w * d1;
      }
    }
  };
  if (lo < hi) {
    TileItem m0 = fetch(lo), m1 = fetch(lo + U);
    float g0[U], o0[U], g1[U], o1[U];
    load(m0, g0, o0);
    for (int j = lo;; j += 2 * U) {
      const TileItem m2 = fetch(j + 2 * U);
      load(m1, g1, o1);
      consume(j, m0, g0, o0);
      if (j + U >= hi) break;
      m0 = fetch(j + 3 * U);
      load(m2, g0, o0);
      consume(j + U, m1, g1, o1);
      if (j + 2 * U >= hi) break;
      m1 = m0;
      m0 = m2;
      // (g0, o0) hold batch j + 2U (m0), m1 the batch after it
    }
  }
  flush();
  if (meta >= 0) {                                 // a split tile's part: its pool slot
    float* ps = pool + (size_t)meta * PT2 * POSE_MAXC;
#pragma unroll
    for (int p = 0; p < PT2; ++p) {
      ps[p * POSE_MAXC + lane] = acc_l[p * ROW + lane];
      ps[p * POSE_MAXC + K1G_CV + lane] = acc_l[p * ROW + K1G_CV + lane];
    }
    return;
  }
  const int tx = tile % ntx, ty = tile / ntx;
  float* db = dP + (size_t)bc * hw * ROW;
#pragma unroll
  for (int p = 0; p < PT2; ++p) {
    const int x = tx * PT + p % PT, y = ty * PT + p / PT;
    if (x >= d.w || y >= d.h) continue;
    float* dst = db + ((size_t)y * d.w + x) * ROW;
    dst[lane] = acc_l[p * ROW + lane];
    dst[K1G_CV + lane] = acc_l[p * ROW + K1G_CV + lane];
  }
}

// split tiles of the K1 gather: the S part slots summed in part order (thread = (tile row, d P
// channel): all PT rows' slot loads in one round)
constexpr int K1C_THREADS = PT * 2 * K1G_CV;
__global__ __launch_bounds__(K1C_THREADS) void fuse_depth_combine_k(vfd_voxel_desc d, const int4* __restrict__ combos,
                                                                    const int* __restrict__ ctrl,
                                                                    const float* __restrict__ pool, float* __restrict__ dP) {
  constexpr int ROW = 2 * K1G_CV;
  const int nt = tiles_x(d) * tiles_y(d), ntx = tiles_x(d);
  const int hw = d.h * d.w;
  const int ch = threadIdx.x % ROW, py = threadIdx.x / ROW;
  const int ncombo = ctrl[1];
  for (int k = blockIdx.x; k < ncombo; k += gridDim.x) {
    const int4 cb = combos[k];
    const int bc = cb.x / nt, tile = cb.x % nt;
    const int x0 = (tile % ntx) * PT, y = (tile / ntx) * PT + py;
    if (y >= d.h) continue;
    const float* p0 = pool + (size_t)cb.y * PT2 * POSE_MAXC + ch;
    float* db = dP + (size_t)bc * hw * ROW + ch;
    // absent parts re-read the last slot and add +0: every load unconditional, summed in part order
    float v[PT][PBW_MAXS];
#pragma unroll
    for (int px = 0; px < PT; ++px)
#pragma unroll
      for (int s2 = 0; s2 < PBW_MAXS; ++s2)
        v[px][s2] = p0[((size_t)min(s2, cb.z - 1) * PT2 + py * PT + px) * POSE_MAXC];
#pragma unroll
    for (int px = 0; px < PT; ++px) {
      float a = v[px][0];
#pragma unroll
      for (int s2 = 1; s2 < PBW_MAXS; ++s2) a += (s2 < cb.z ? 1.f : 0.f) * v[px][s2];
      if (x0 + px < d.w) db[((size_t)y * d.w + x0 + px) * ROW] = a;
    }
  }
}

// K3 geometry (Tri, frustum_sample, tri_index, corner_offset): vfd_common.h

// ------------------------------------------------------------------------------ K3 forward
// Frustum samples -> trilinear gather from the channels-last voxel grid (K1's output), written
// into the channels-last input of reduce_dim's first conv: out[bc][y'][x'][d*Cv + c] (NHWC,
// depth-major channels; the conv weight is permuted to match).  Samples are numbered
// s = pixel * D + depth, the output order, so consecutive samples write consecutive Cv-rows.
// A workgroup owns 64 consecutive samples: one thread per sample computes the cell and weights
// into LDS, then each wave processes its 16 samples four at a time with lanes = (sample,
// channel quad): every corner read and every output store is one float4 per lane (a 256-B row
// per 16 lanes), and the per-sample index math runs on vector lanes (no scalar-unit loop).
constexpr int VP_S = 64;        // samples per workgroup

struct TriLds {
  int base[VP_S];               // voxel index of corner 0 (may be out of range; see in)
  unsigned in[VP_S];
  float w[VP_S][8];
};

__device__ __forceinline__ void tri_to_lds(const vfd_voxel_desc& d, TriLds& tl, int j, const Tri& t) {
  tl.base[j] = (t.z0 * d.Y + t.y0) * d.X + t.x0;
  tl.in[j] = t.in;
#pragma unroll
  for (int k = 0; k < 8; ++k) tl.w[j][k] = t.w[k];
}


template <int CV>
__global__ __launch_bounds__(256) void voxel_project_fwd_k(vfd_voxel_desc d, const float* __restrict__ vox,
                                                           const float* __restrict__ invK,
                                                           const float* __restrict__ E,
                                                           float* __restrict__ out) {
  constexpr int QPS = CV / 4;           // float4 quads per sample row
  constexpr int SPI = 64 / QPS;         // samples per wave instruction
  __shared__ TriLds tl;
  const int S = d.h * d.w * d.D;        // samples per (batch, camera)
  // XCD-aware numbering: XCD k takes the contiguous task range [k*per, (k+1)*per) — the
  // workgroups resident on one XCD sweep neighbouring rays, which read one wedge of the grid
  const int nchunk = (S + VP_S - 1) / VP_S;
  const int ntask = nchunk * d.B * d.N;
  const int per = gridDim.x / 8;
  const int task = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (task >= ntask) return;
  const int bc = task / nchunk, b = bc / d.N;
  const int s0 = (task % nchunk) * VP_S;
  if (threadIdx.x < VP_S) {
    const int sl = s0 + threadIdx.x;
    Tri t;
    t.in = 0;
    t.x0 = t.y0 = t.z0 = 0;
    if (sl < S) {
      const int p = sl / d.D, di = sl % d.D;
      t = frustum_sample(d, invK + bc * 16, E + bc * 16, p % d.w, p / d.w, d.dbins[di]);
    }
    tri_to_lds(d, tl, threadIdx.x, t);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int grp = lane / QPS, q = lane % QPS;
  const int V = d.X * d.Y * d.Z;
  const float4* vb = reinterpret_cast<const float4*>(vox + (size_t)b * V * CV) + q;
  const int P = d.pad_out ? 2 : 0;
  const int ho = d.h + P, wo = d.w + P;
  float4* ob = reinterpret_cast<float4*>(out + (size_t)bc * ho * wo * d.D * CV) + q;
  constexpr int SPW = VP_S / 4;          // samples per wave
#pragma unroll
  for (int it = 0; it < (SPW + SPI - 1) / SPI; ++it) {
    if (it * SPI + grp >= SPW) break;     // (only when a wave instruction spans > SPW samples)
    const int j = wv * SPW + it * SPI + grp;                  // sample within the workgroup
    const int sl = s0 + j;
    const unsigned in = tl.in[j];
    const int base = tl.base[j];
    // branch-free: every corner is loaded (out-of-range ones from voxel 0 with weight 0, which
    // adds +0: the reference's sum over in-range corners, same order)
    float4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const bool ok = (in >> k & 1u) != 0u;
      v[k] = vb[(size_t)(ok ? base + corner_offset(d, k) : 0) * QPS];
    }
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float w = (in >> k & 1u) ? tl.w[j][k] : 0.f;
      acc.x += v[k].x * w;
      acc.y += v[k].y * w;
      acc.z += v[k].z * w;
      acc.w += v[k].w * w;
    }
    if (sl < S) {
      const int p = sl / d.D, di = sl % d.D;
      const int px = p % d.w, py = p / d.w;
      int rows[3], cols[3], nr, nc;
      pad_sets(py, d.h, d.pad_out, rows, &nr);
      pad_sets(px, d.w, d.pad_out, cols, &nc);
      for (int r = 0; r < nr; ++r)
        for (int c2 = 0; c2 < nc; ++c2)
          ob[(((size_t)rows[r] * wo + cols[c2]) * d.D + di) * QPS] = acc;
    }
  }
}

// ------------------------------------------------------------------------------ K3 backward
// The transpose of the trilinear gather: every frustum sample adds w_k * g to the 8 corners of
// its voxel cell.  f32 atomics run at one chip-wide rate (~1.3 TB/s of added bytes, and LDS
// float atomics at ~3 cycles per lane), so the backward is organised as an owner-computes
// accumulation with no float atomics on the common path:
//   vpb_count_k / vpb_fill_k  counting sort of the samples by cell (extended grid of
//                             (X+1)(Y+1)(Z+1) cells, corner 0 in [-1, X-1] ...): one 16-B
//                             entry {ix, iy, iz, sample} per in-range sample, cells contiguous
//                             in x;
//   vpb_brick_k / vpb_tasks_k voxel bricks of 8x8x4; a brick's wave for voxel layer zl owns the
//                             samples of the 2 x 9 cell rows that touch that layer (18
//                             contiguous entry ranges); bricks whose heaviest layer has more
//                             than VB_S samples are split into parts (their voxels zeroed and
//                             flushed with atomics);
//   vpb_main_k                one workgroup per task, lanes = channels, 64 KB LDS brick
//                             accumulator: each wave reads its samples' gradient rows (reflect
//                             copies folded), merges runs of one cell in registers and flushes
//                             the cell's 4 corners of its own layer into LDS with plain
//                             read-add-write (no other wave writes that layer); the brick is
//                             then written with plain stores.
#ifndef VFD_VPB_PQ
#define VFD_VPB_PQ 8
#endif
constexpr int VB_X = 8, VB_Y = 4;                  // voxel tile (one z layer) per wave task
// One wave per voxel layer (vpb_main_k), each reading the two cell layers around it.  (A z-walk
// form — one wave sweeping a brick column, each gradient row read once for both voxel layers it
// feeds — measured 315-370 us vs 207 us at config 2: its second LDS layer slot halves the resident
// waves of this latency-bound loop; DESIGN.md section 4.  Removed from the library, in git history.)
#ifndef VFD_VPB_LG
#define VFD_VPB_LG 2          // 4 and 5 measured slower (219, 263 us vs 209 us at config 2)
#endif
constexpr int VB_LG = VFD_VPB_LG;                  // voxel layers (waves) per workgroup task
constexpr int VB_RY = VB_Y + 1, VB_NSEG = 2 * VB_RY;   // cell rows per layer, entry ranges per tile
#ifndef VFD_VPB_S
#define VFD_VPB_S 1024
#endif
constexpr int VB_S = VFD_VPB_S;                    // samples per task part
constexpr int VB_SCAN = 4096;                      // cells per block of the first scan level

struct VpbGeom {
  int CX, CY, CZ, ncell;                           // extended cell grid per batch
  int nbx, nby, ntile;                             // tiles per batch: nbx * nby * ceil(Z / 2) layer pairs
};
__host__ __device__ __forceinline__ VpbGeom vpb_geom(const vfd_voxel_desc& d) {
  VpbGeom g;
  g.CX = d.X + 1;
  g.CY = d.Y + 1;
  g.CZ = d.Z + 1;
  g.ncell = g.CX * g.CY * g.CZ;
  g.nbx = (d.X + VB_X - 1) / VB_X;
  g.nby = (d.Y + VB_Y - 1) / VB_Y;
  g.ntile = g.nbx * g.nby * ((d.Z + VB_LG - 1) / VB_LG);
  return g;
}

// Tile tl of a batch -> brick origin (xb, yb) and layer pair zp.  Layer pairs are the fastest
// index: the tasks of one brick column are consecutive, so (with vpb_main_k's per-XCD task
// ranges) neighbouring layer pairs run at about the same time on one XCD and the cell layer each
// pair shares with the next (2 zp + 1) is fetched into that XCD's L2 once.
#ifndef VFD_VPB_ZFAST
#define VFD_VPB_ZFAST 1
#endif
#ifndef VFD_VPB_XCDQ
#define VFD_VPB_XCDQ 0          // 1: per-XCD task ranges + stealing, 2: static per XCD (both measured slower)
#endif
__device__ __forceinline__ void vpb_tile_pos(const vfd_voxel_desc& d, const VpbGeom& g, int tl, int* xb, int* yb,
                                             int* zp) {
#if VFD_VPB_ZFAST
  const int nzp = (d.Z + VB_LG - 1) / VB_LG;
  *zp = tl % nzp;
  const int r = tl / nzp;
  *xb = (r % g.nbx) * VB_X;
  *yb = (r / g.nbx) * VB_Y;
#else
  *xb = (tl % g.nbx) * VB_X;
  *yb = ((tl / g.nbx) % g.nby) * VB_Y;
  *zp = tl / (g.nbx * g.nby);
#endif
}

// continuous grid coordinates of a frustum sample (the first half of frustum_sample)
__device__ __forceinline__ void frustum_coords(const vfd_voxel_desc& d, const float* __restrict__ iK,
                                               const float* __restrict__ E, int px, int py, float dep,
                                               float* ix, float* iy, float* iz) {
  float fx = (float)px, fy = (float)py;
  float r0 = iK[0] * fx + iK[1] * fy + iK[2];
  float r1 = iK[4] * fx + iK[5] * fy + iK[6];
  float r2 = iK[8] * fx + iK[9] * fy + iK[10];
  float p0 = dep * r0, p1 = dep * r1, p2 = dep * r2;
  float w0 = E[0] * p0 + E[1] * p1 + E[2] * p2 + E[3];
  float w1 = E[4] * p0 + E[5] * p1 + E[6] * p2 + E[7];
  float w2 = E[8] * p0 + E[9] * p1 + E[10] * p2 + E[11];
  float gx = (w0 - d.str[0]) / d.len[0] * 2.f - 1.f;
  float gy = (w1 - d.str[1]) / d.len[1] * 2.f - 1.f;
  float gz = (w2 - d.str[2]) / d.len[2] * 2.f - 1.f;
  *ix = unnorm_ac(gx, d.X);
  *iy = unnorm_ac(gy, d.Y);
  *iz = unnorm_ac(gz, d.Z);
}

// extended-grid cell of a sample whose cell has at least one in-range corner, else -1
__device__ __forceinline__ int vpb_cell(const vfd_voxel_desc& d, const VpbGeom& g, float ix, float iy, float iz) {
  if (!(finitef(ix) && finitef(iy) && finitef(iz))) return -1;
  const float fx0 = floorf(ix), fy0 = floorf(iy), fz0 = floorf(iz);
  if (!(fx0 >= -1.f && fx0 <= (float)(d.X - 1) && fy0 >= -1.f && fy0 <= (float)(d.Y - 1) && fz0 >= -1.f &&
        fz0 <= (float)(d.Z - 1)))
    return -1;
  return (((int)fz0 + 1) * g.CY + ((int)fy0 + 1)) * g.CX + ((int)fx0 + 1);
}

// Sort order inside the count / fill kernels: sl = depth * hw + pixel (pixels fastest, so a
// wave's lanes are neighbouring pixels at one depth and often share a cell near the camera: the
// lanes of a run of equal cells take their ranks with ONE counter atomic, issued by the run head).
// The entry's sample id is s = (bc * hw + pixel) * D + depth (the order of the gradient rows).
__device__ __forceinline__ void vpb_count(const vfd_voxel_desc& d, const float* __restrict__ invK,
                                          const float* __restrict__ E, int* __restrict__ cnt,
                                          int* __restrict__ rank, int bc, int blk) {
  const VpbGeom g = vpb_geom(d);
  const int b = bc / d.N;
  const int hw = d.h * d.w, hwD = hw * d.D;
  const int sl = blk * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  int c = -1;
  if (sl < hwD) {
    const int di = sl / hw, p = sl % hw;
    float ix, iy, iz;
    frustum_coords(d, invK + bc * 16, E + bc * 16, p % d.w, p / d.w, d.dbins[di], &ix, &iy, &iz);
    c = vpb_cell(d, g, ix, iy, iz);
  }
  const int prev = __shfl_up(c, 1, 64);
  const bool head = lane == 0 || c != prev;
  const unsigned long long hm = __ballot(head);
  const unsigned long long le = lane == 63 ? ~0ull : ((2ull << lane) - 1);     // lanes <= lane
  const int myhead = 63 - __clzll(hm & le);
  const unsigned long long after = hm & ~le;
  const int next = after ? __ffsll((long long)after) - 1 : 64;
  int r = 0;
  if (head && c >= 0) r = atomicAdd(cnt + (size_t)b * g.ncell + c, next - lane);
  r = __shfl(r, myhead, 64) + lane - myhead;
  if (sl < hwD) rank[(size_t)bc * hwD + sl] = c < 0 ? -1 : r;
}

// first scan level: exclusive prefix of VB_SCAN counts per block (16 per thread), block totals
__global__ __launch_bounds__(256) void vpb_scan1_k(const int* __restrict__ cnt, int n, int* __restrict__ ptr,
                                                   int* __restrict__ bsum) {
  __shared__ int wsum[4];
  const int base = blockIdx.x * VB_SCAN + threadIdx.x * 16;
  int v[16], run = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    v[i] = base + i < n ? cnt[base + i] : 0;
    run += v[i];
  }
  // inclusive wave scan of the per-thread totals
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int inc = run;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int t = __shfl_up(inc, off, 64);
    if (lane >= off) inc += t;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  int woff = 0;
  for (int k = 0; k < wv; ++k) woff += wsum[k];
  int ex = woff + inc - run;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (base + i < n) ptr[base + i] = ex;
    ex += v[i];
  }
  if (threadIdx.x == 255) bsum[blockIdx.x] = woff + inc;
}

// second level: one workgroup, exclusive prefix of the block totals; boff[nblk] = grand total
__global__ __launch_bounds__(1024) void vpb_scan2_k(const int* __restrict__ bsum, int nblk, int* __restrict__ boff) {
  __shared__ int part[1024];
  const int t = threadIdx.x;
  const int chunk = (nblk + 1023) / 1024;
  const int c0 = min(nblk, t * chunk), c1 = min(nblk, c0 + chunk);
  int local = 0;
  for (int i = c0; i < c1; ++i) local += bsum[i];
  part[t] = local;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = part[t] - local;
  for (int i = c0; i < c1; ++i) {
    boff[i] = run;
    run += bsum[i];
  }
  if (t == 1023) boff[nblk] = part[t];
}

// start of cell i's entries (i == n: the total)
__device__ __forceinline__ int vpb_ptr(const int* __restrict__ ptr, const int* __restrict__ boff, int n, int i) {
  return i < n ? ptr[i] + boff[i / VB_SCAN] : boff[(n + VB_SCAN - 1) / VB_SCAN];
}

__device__ __forceinline__ int vpb_fold_slot(const vfd_voxel_desc& d, int px, int py);

// entry = {ix, iy, iz, row}: row = the sample's gradient row (CV floats): bit 31 clear = row of
// d_out, set = row of fbz (row 0 = a zero row, 1 + ... = folded rows of pixels with reflect copies)
__global__ __launch_bounds__(256) void vpb_fill_k(vfd_voxel_desc d, const float* __restrict__ invK,
                                                  const float* __restrict__ E, const int* __restrict__ rank,
                                                  const int* __restrict__ ptr, const int* __restrict__ boff,
                                                  float4* __restrict__ entries) {
  const VpbGeom g = vpb_geom(d);
  const int bc = blockIdx.y, b = bc / d.N;
  const int hw = d.h * d.w, hwD = hw * d.D;
  const int sl = blockIdx.x * blockDim.x + threadIdx.x;
  if (sl >= hwD) return;
  const int r = rank[(size_t)bc * hwD + sl];
  if (r < 0) return;
  const int di = sl / hw, p = sl % hw;
  const int px = p % d.w, py = p / d.w;
  float ix, iy, iz;
  frustum_coords(d, invK + bc * 16, E + bc * 16, px, py, d.dbins[di], &ix, &iy, &iz);
  const int c = vpb_cell(d, g, ix, iy, iz);
  const int n = d.B * g.ncell;
  const int Pd = d.pad_out ? 1 : 0;
  const int fs = d.pad_out == 1 ? vpb_fold_slot(d, px, py) : -1;   // pad_out 2: d_out arrives folded
  const unsigned row = fs >= 0 ? 0x80000000u | (unsigned)(1 + (bc * 2 * (d.w + d.h) + fs) * d.D + di)
                               : (unsigned)(((bc * (d.h + 2 * Pd) + py + Pd) * (d.w + 2 * Pd) + px + Pd) * d.D + di);
  entries[vpb_ptr(ptr, boff, n, b * g.ncell + c) + r] = make_float4(ix, iy, iz, __uint_as_float(row));
}

// Deterministic mode: the count kernel ranks a cell's samples by atomic arrival.  vpb_order_k
// re-ranks every filled entry within its cell by its gradient row (one row per sample: unique)
// and writes that rank back to the sample's slot of `rank`; a second vpb_fill_k then places the
// entries in that order.
__device__ __forceinline__ int vpb_row_sample(const vfd_voxel_desc& d, unsigned row, int* bc) {
  const int Pd = d.pad_out ? 1 : 0, hw = d.h * d.w;
  int px, py, di;
  if (row >> 31) {
    const int r = (int)(row & 0x7FFFFFFFu) - 1, nfs = 2 * (d.w + d.h);
    di = r % d.D;
    const int t = r / d.D, fs = t % nfs;
    *bc = t / nfs;
    if (fs < d.w) { px = fs; py = 1; }
    else if (fs < 2 * d.w) { px = fs - d.w; py = d.h - 2; }
    else if (fs < 2 * d.w + d.h) { px = 1; py = fs - 2 * d.w; }
    else { px = d.w - 2; py = fs - 2 * d.w - d.h; }
  } else {
    const int r = (int)row;
    di = r % d.D;
    const int t = r / d.D, W2 = d.w + 2 * Pd, H2 = d.h + 2 * Pd;
    px = t % W2 - Pd;
    py = (t / W2) % H2 - Pd;
    *bc = t / (W2 * H2);
  }
  return di * hw + py * d.w + px;                   // sl of the count / fill kernels
}

__global__ __launch_bounds__(256) void vpb_order_k(vfd_voxel_desc d, const int* __restrict__ ptr,
                                                   const int* __restrict__ boff, const float4* __restrict__ entries,
                                                   int* __restrict__ rank) {
  const VpbGeom g = vpb_geom(d);
  const int n = d.B * g.ncell;
  const int total = vpb_ptr(ptr, boff, n, n);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  int lo = 0, hi = n;                               // last cell c with start(c) <= i
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (vpb_ptr(ptr, boff, n, mid) <= i) lo = mid; else hi = mid;
  }
  const int s0 = vpb_ptr(ptr, boff, n, lo), s1 = vpb_ptr(ptr, boff, n, lo + 1);
  const unsigned key = __float_as_uint(entries[i].w);
  int r = 0;
  for (int j = s0; j < s1; ++j) r += __float_as_uint(entries[j].w) < key ? 1 : 0;
  int bc;
  const int sl = vpb_row_sample(d, key, &bc);
  rank[(size_t)bc * d.h * d.w * d.D + sl] = r;
}

// Reflect-pad fold (pad_sets): the gradient of map pixel (px, py) is the sum of its copies in the
// padded d_out.  Only pixels with a second copy (py in {1, h-2} or px in {1, w-2}) are folded,
// into fb[bc][slot][D][CV]; slot = px (py == 1), w + px (py == h-2), 2w + py (px == 1),
// 2w + h + py (px == w-2), first match wins.
__device__ __forceinline__ int vpb_fold_slot(const vfd_voxel_desc& d, int px, int py) {
  if (py == 1) return px;
  if (py == d.h - 2) return d.w + px;
  if (px == 1) return 2 * d.w + py;
  if (px == d.w - 2) return 2 * d.w + d.h + py;
  return -1;
}

template <int CV>
__device__ __forceinline__ void vpb_fold(const vfd_voxel_desc& d, const float* __restrict__ dout,
                                         float* __restrict__ fb, int fblk) {
  const int nsl = 2 * (d.w + d.h);
  const int bc = fblk / nsl, slot = fblk % nsl;
  int px, py;
  if (slot < d.w) { px = slot; py = 1; }
  else if (slot < 2 * d.w) { px = slot - d.w; py = d.h - 2; }
  else if (slot < 2 * d.w + d.h) { px = 1; py = slot - 2 * d.w; }
  else { px = d.w - 2; py = slot - 2 * d.w - d.h; }
  if (vpb_fold_slot(d, px, py) != slot) return;          // owned by an earlier slot
  const int wo = d.w + 2, ho = d.h + 2;
  int rows[3], cols[3], nr, nc;
  pad_sets(py, d.h, true, rows, &nr);
  pad_sets(px, d.w, true, cols, &nc);
  const size_t rl = (size_t)d.D * CV;
  const float4* src[9];
  int ns = 0;
  for (int a = 0; a < nr; ++a)
    for (int c2 = 0; c2 < nc; ++c2)
      src[ns++] = reinterpret_cast<const float4*>(dout + (((size_t)bc * ho + rows[a]) * wo + cols[c2]) * rl);
  float4* dst = reinterpret_cast<float4*>(fb + ((size_t)bc * nsl + slot) * rl);
  for (int i = threadIdx.x; i < (int)(rl / 4); i += blockDim.x) {
    float4 s = src[0][i];
    for (int k = 1; k < ns; ++k) {
      const float4 v = src[k][i];
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
    dst[i] = s;
  }
}

// plan phase: count samples per cell (latency-bound returning atomics)
__global__ __launch_bounds__(256) void vpb_count_k(vfd_voxel_desc d, const float* __restrict__ invK,
                                                   const float* __restrict__ E, int* __restrict__ cnt,
                                                   int* __restrict__ rank, int cpb) {
  vpb_count(d, invK, E, cnt, rank, blockIdx.x / cpb, blockIdx.x % cpb);
}

// backward phase, one launch: blocks [0, nf) fold the reflect copies of d_out (streaming), blocks
// [nf, nf + nb) zero the voxels of split tiles (their parts add with atomics), block nf + nb
// resets main's work counter
template <int CV>
__global__ __launch_bounds__(256) void vpb_fold_zero_k(vfd_voxel_desc d, const float* __restrict__ dout,
                                                       float* __restrict__ fb, int nf, const int* __restrict__ parts,
                                                       int nb, int* __restrict__ ctrl, float* __restrict__ dvox) {
  const int blk = blockIdx.x;
  if (blk < nf) {
    vpb_fold<CV>(d, dout, fb, blk);
    return;
  }
  const int tile = blk - nf;
  if (tile >= nb) {
    if (threadIdx.x < 8) ctrl[8 + threadIdx.x] = 0;    // vpb_main_k's per-XCD work counters
    return;
  }
  if (parts[tile] <= 1) return;
  const VpbGeom g = vpb_geom(d);
  const int b = tile / g.ntile, tl = tile % g.ntile;
  int xb, yb, zp;
  vpb_tile_pos(d, g, tl, &xb, &yb, &zp);
  const int V = d.X * d.Y * d.Z;
  constexpr int QPV = CV / 4;
  for (int i = threadIdx.x; i < VB_LG * VB_X * VB_Y * QPV; i += blockDim.x) {
    const int q = i % QPV, v = (i / QPV) % (VB_X * VB_Y), zl = VB_LG * zp + i / (QPV * VB_X * VB_Y);
    const int x = xb + v % VB_X, y = yb + v / VB_X;
    if (x < d.X && y < d.Y && zl < d.Z)
      reinterpret_cast<float4*>(dvox + ((size_t)b * V + (zl * d.Y + y) * d.X + x) * CV)[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// entry range of cell row (z0, y0) of brick column [xb - 1, xb + 7] (clipped to the grid)
__device__ __forceinline__ void vpb_segment(const vfd_voxel_desc& d, const VpbGeom& g, const int* __restrict__ ptr,
                                            const int* __restrict__ boff, int b, int z0, int y0, int xb, int* s0,
                                            int* s1) {
  if (y0 < -1 || y0 > d.Y - 1 || z0 < -1 || z0 > d.Z - 1) {
    *s0 = *s1 = 0;
    return;
  }
  const int n = d.B * g.ncell;
  const int base = b * g.ncell + ((z0 + 1) * g.CY + (y0 + 1)) * g.CX;
  *s0 = vpb_ptr(ptr, boff, n, base + xb);
  *s1 = vpb_ptr(ptr, boff, n, base + min(xb + VB_X, d.X) + 1);
}

// Entry range k (< VB_NSEG) of the wave for layer zl = VB_LG zp + w of a layer-group tile: the
// cell layers of zl are z0 = zl - 1 (its samples weigh in with dz = 1) and z0 = zl (dz = 0); each
// is shared with a neighbouring wave.  Even waves read z0 = zl first, odd waves z0 = zl - 1 first,
// so waves (2k, 2k+1) read their shared layer in their first halves and (2k+1, 2k+2) in their
// second halves: roughly at the same time, one L2 fetch for both.  Inside a group a cell layer is
// fetched once, so a group of VB_LG layers reads VB_LG + 1 cell layers.
__device__ __forceinline__ int vpb_seg_z0(int zp, int w, int k) {
  const int zl = VB_LG * zp + w;
  const bool own_first = (w & 1) == 0;
  return (k < VB_RY) == own_first ? zl : zl - 1;
}

// per layer-pair tile: samples of each layer's wave -> number of parts (split tiles are zeroed by
// vpb_fold_zero_k in the backward phase).  grid = B * ntile, block = one wave
__global__ __launch_bounds__(64) void vpb_tile_k(vfd_voxel_desc d, const int* __restrict__ ptr,
                                                 const int* __restrict__ boff, int* __restrict__ parts) {
  const VpbGeom g = vpb_geom(d);
  const int tile = blockIdx.x, lane = threadIdx.x;
  const int b = tile / g.ntile, tl = tile % g.ntile;
  int xb, yb, zp;
  vpb_tile_pos(d, g, tl, &xb, &yb, &zp);
  static_assert(VB_LG * VB_NSEG <= 64, "one lane per entry range");
  int n = 0, wl = -1;
  if (lane < VB_LG * VB_NSEG) {
    const int w = lane / VB_NSEG, k = lane % VB_NSEG;
    if (VB_LG * zp + w < d.Z) {
      int s0, s1;
      vpb_segment(d, g, ptr, boff, b, vpb_seg_z0(zp, w, k), yb - 1 + k % VB_RY, xb, &s0, &s1);
      n = s1 - s0;
      wl = w;
    }
  }
  int nmax = 0;
#pragma unroll
  for (int w = 0; w < VB_LG; ++w) nmax = max(nmax, wave_sum(wl == w ? n : 0));
  // deterministic mode: no split tiles (their parts would add with atomics)
  const int np = d.deterministic ? 1 : max(1, (nmax + VB_S - 1) / VB_S);
  if (lane == 0) parts[tile] = np;
}

// one workgroup: task list (int2 {tile, part | nparts << 16}), task count, main's work counter
__global__ __launch_bounds__(1024) void vpb_tasks_k(const int* __restrict__ parts, int nb, int2* __restrict__ tasks,
                                                    int* __restrict__ ctrl) {
  __shared__ int part[1024];
  const int t = threadIdx.x;
  const int chunk = (nb + 1023) / 1024;
  const int c0 = min(nb, t * chunk), c1 = min(nb, c0 + chunk);
  int local = 0;
  for (int i = c0; i < c1; ++i) local += parts[i];
  part[t] = local;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = part[t] - local;
  for (int i = c0; i < c1; ++i) {
    const int np = parts[i];
    for (int q = 0; q < np; ++q) tasks[run + q] = make_int2(i, q | (np << 16));
    run += np;
  }
  if (t == 1023) ctrl[0] = part[t];                 // tasks
  if (t < 8) ctrl[8 + t] = 0;                         // per-XCD work counters of vpb_main_k
}

// One wave = one independent worker: it takes tile tasks from the counter, accumulates its tile
// in a private 16 KB LDS slab and writes it out (plain stores, or atomics for split tiles).
template <int CV>
__global__ __launch_bounds__(64 * VB_LG) void vpb_main_k(vfd_voxel_desc d, const int* __restrict__ ptr,
                                                  const int* __restrict__ boff, const float4* __restrict__ entries,
                                                  const int2* __restrict__ tasks, int* __restrict__ ctrl,
                                                  const float* __restrict__ dout, const float* __restrict__ fbz,
                                                  float* __restrict__ dvox) {
  constexpr int LAYER = VB_Y * VB_X * 64;
  __shared__ float lacc_l[VB_LG][LAYER + 64];      // per wave: its layer + one scratch row (masked corners)
  __shared__ int task_l;
  const VpbGeom g = vpb_geom(d);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int cl = lane < CV ? lane : 0;
  const int V = d.X * d.Y * d.Z;
  const int ntask = ctrl[0];
  float* lacc = lacc_l[wv];
  float* trash = lacc + LAYER;
  // Work queues: the task list is cut into 8 contiguous ranges, one per XCD (workgroups are dealt
  // round-robin to the XCDs, so blockIdx % 8 names this one's); a worker drains its XCD's range in
  // order, then steals from the others.  Counters past a range's end are harmless.
  const int xcd = blockIdx.x & 7;
  for (int iter = 0;; ++iter) {
    __syncthreads();
    if (threadIdx.x == 0) {
      int tk = -1;
#if VFD_VPB_XCDQ == 0
      tk = atomicAdd(ctrl + 8, 1);
      if (tk >= ntask) tk = -1;
#elif VFD_VPB_XCDQ == 2
      {   // static: this XCD's range, round-robin over its workgroups (no atomics)
        const int lo = (int)((long long)ntask * xcd / 8), hi = (int)((long long)ntask * (xcd + 1) / 8);
        const int i = lo + (int)(blockIdx.x >> 3) + iter * (int)(gridDim.x >> 3);
        tk = i < hi ? i : -1;
      }
#else
      for (int k = 0; k < 8; ++k) {
        const int qq = (xcd + k) & 7;
        const int lo = (int)((long long)ntask * qq / 8), hi = (int)((long long)ntask * (qq + 1) / 8);
        if (lo >= hi) continue;
        const int i = atomicAdd(ctrl + 8 + qq, 1);
        if (lo + i < hi) {
          tk = lo + i;
          break;
        }
      }
#endif
      task_l = tk;
    }
    for (int i = lane; i < LAYER / 4; i += 64) reinterpret_cast<float4*>(lacc)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    __syncthreads();
    const int t = task_l;
    if (t < 0) break;
    const int2 tk = tasks[t];
    const int tile = tk.x, part = tk.y & 0xFFFF, np = tk.y >> 16;
    const int b = tile / g.ntile, tl = tile % g.ntile;
    int xb, yb, zp;
    vpb_tile_pos(d, g, tl, &xb, &yb, &zp);
    const int zl = VB_LG * zp + wv;                  // this wave's voxel layer
    if (zl < d.Z) {
      // the wave's entry ranges (lanes 0 .. VB_NSEG-1) and their running offsets
      int s0 = 0, s1 = 0;
      if (lane < VB_NSEG) vpb_segment(d, g, ptr, boff, b, vpb_seg_z0(zp, wv, lane), yb - 1 + lane % VB_RY, xb, &s0, &s1);
      const int len = s1 - s0;
      int inc = len;
#pragma unroll
      for (int off = 1; off < 32; off <<= 1) {
        const int tt = __shfl_up(inc, off, 64);
        if (lane >= off) inc += tt;
      }
      const int total = __builtin_amdgcn_readlane(inc, VB_NSEG - 1);
      const int lo = (int)((long long)total * part / np), hi = (int)((long long)total * (part + 1) / np);
      // entry of list position gi (clamped into [lo, hi): the load is unconditional, so it stays
      // in flight behind the row loads instead of forcing a wait inside a divergent branch)
      auto entry_of = [&](int gi) {
        gi = min(gi, hi - 1);
        int seg = 0;
#pragma unroll
        for (int k = 0; k < VB_NSEG - 1; ++k) seg += gi >= __builtin_amdgcn_readlane(inc, k) ? 1 : 0;
        const int ss = __shfl(s0, seg, 64), ex = __shfl(inc - len, seg, 64);
        return entries[ss + gi - ex];
      };
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
      int cur = -1;                  // current cell key (wave-uniform)
      unsigned cmask = 0;            // its in-brick, in-grid corner mask
      // branch-free: masked corners go to the wave's scratch row (their sums are exactly 0)
      auto flush = [&]() {
        const int lx = (cur & 15) - 1, ly = ((cur >> 4) & 15) - 1;
        float* r0 = lacc + (ly * VB_X + lx) * 64;
        float* p0 = (cmask & 1u) ? r0 : trash;
        float* p1 = (cmask & 2u) ? r0 + 64 : trash;
        float* p2 = (cmask & 4u) ? r0 + VB_X * 64 : trash;
        float* p3 = (cmask & 8u) ? r0 + VB_X * 64 + 64 : trash;
        const float v0 = p0[lane], v1 = p1[lane], v2 = p2[lane], v3 = p3[lane];
        p0[lane] = v0 + a0;
        p1[lane] = v1 + a1;
        p2[lane] = v2 + a2;
        p3[lane] = v3 + a3;
        a0 = a1 = a2 = a3 = 0.f;
      };
      // Software pipeline over half-batches of 32 samples: the rows of the next half are in
      // flight while the current half is accumulated (<= 64 loads outstanding: vmcnt's range).
      struct Prm {
        int key, m;
        float w0, w1, w2, w3;
        unsigned row;
      };
      auto setup = [&](const float4& e, int g0) {
        Prm q;
        const bool valid = g0 + lane < hi;
        const float fx0 = floorf(e.x), fy0 = floorf(e.y), fz0 = floorf(e.z);
        const float ax0 = fx0 + 1.f - e.x, ax1 = e.x - fx0, ay0 = fy0 + 1.f - e.y, ay1 = e.y - fy0;
        const int x0 = (int)fx0, y0 = (int)fy0, z0 = (int)fz0;
        const int dz = valid ? zl - z0 : 0;
        const float az = dz ? e.z - fz0 : fz0 + 1.f - e.z;
        // ATen trilinear weights (ax[dx] * ay[dy]) * az[dz], as in frustum_sample
        q.w0 = ax0 * ay0 * az;
        q.w1 = ax1 * ay0 * az;
        q.w2 = ax0 * ay1 * az;
        q.w3 = ax1 * ay1 * az;
        const bool xin0 = x0 >= max(xb, 0), xin1 = x0 + 1 < min(xb + VB_X, d.X);
        const bool yin0 = y0 >= max(yb, 0), yin1 = y0 + 1 < min(yb + VB_Y, d.Y);
        q.m = valid ? (xin0 && yin0 ? 1 : 0) | (xin1 && yin0 ? 2 : 0) | (xin0 && yin1 ? 4 : 0) | (xin1 && yin1 ? 8 : 0)
                    : 0;
        // samples past the end: key -1 (one flush of the open cell, then nothing), a zero row
        q.key = valid ? ((1 - dz) << 8) | ((y0 - yb + 1) << 4) | (x0 - xb + 1) : -1;
        q.row = valid ? __float_as_uint(e.w) : 0x80000000u;     // past the end: the zero row
        return q;
      };
      constexpr int PQ = VFD_VPB_PQ;    // samples per pipeline stage (64 / PQ stages per batch)
      auto load_part = [&](const Prm& q, int h, float* gr) {
#pragma unroll
        for (int j = 0; j < PQ; ++j) {
          const unsigned rj = (unsigned)__builtin_amdgcn_readlane((int)q.row, h * PQ + j);
          const float* src = (rj >> 31) ? fbz : dout;      // wave-uniform: scalar select
          gr[j] = src[(size_t)(rj & 0x7FFFFFFFu) * CV + cl];
        }
      };
      auto process_part = [&](const Prm& q, int h, const float* gr) {
#pragma unroll
        for (int j = 0; j < PQ; ++j) {
          const int jj = h * PQ + j;
          const float gj = gr[j];
          const int kj = __builtin_amdgcn_readlane(q.key, jj);
          if (kj != cur) {
            flush();
            cur = kj;
            cmask = (unsigned)__builtin_amdgcn_readlane(q.m, jj);
          }
          a0 += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q.w0), jj)) * gj;
          a1 += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q.w1), jj)) * gj;
          a2 += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q.w2), jj)) * gj;
          a3 += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q.w3), jj)) * gj;
        }
      };
      if (lo < hi) {
        constexpr int NST = 64 / PQ;
        float4 en = entry_of(lo + lane);
        Prm P = setup(en, lo);
        en = entry_of(lo + 64 + lane);
        float gr[2][PQ];
        load_part(P, 0, gr[0]);
        // every load is unconditional (samples past the end read the zero row): a load under a
        // branch makes the compiler's vmcnt accounting at the join wait for everything
        for (int g0 = lo; g0 < hi; g0 += 64) {
          Prm Pn = P;
#pragma unroll
          for (int st = 0; st < NST; ++st) {
            if (st + 1 < NST) {
              load_part(P, st + 1, gr[(st + 1) & 1]);
            } else {
              Pn = setup(en, g0 + 64);
              en = entry_of(g0 + 128 + lane);
              load_part(Pn, 0, gr[(st + 1) & 1]);
            }
            process_part(P, st, gr[st & 1]);
          }
          P = Pn;
        }
      }
      flush();
    }
    // ---- write the tile: lanes = (voxel, channel quad)
    if (zl < d.Z) {
      constexpr int QPV = CV / 4, VPI = 64 / QPV;
      const int q = lane % QPV, vsub = lane / QPV;
      for (int v0 = 0; v0 < VB_X * VB_Y; v0 += VPI) {
        const int vl = v0 + vsub;
        const int x = xb + vl % VB_X, y = yb + vl / VB_X;
        if (x >= d.X || y >= d.Y) continue;
        const float4 a = *reinterpret_cast<const float4*>(lacc + vl * 64 + q * 4);
        float* dst = dvox + ((size_t)b * V + ((size_t)zl * d.Y + y) * d.X + x) * CV + q * 4;
        if (np == 1) {
          *reinterpret_cast<float4*>(dst) = a;
        } else {
          unsafeAtomicAdd(dst + 0, a.x);
          unsafeAtomicAdd(dst + 1, a.y);
          unsafeAtomicAdd(dst + 2, a.z);
          unsafeAtomicAdd(dst + 3, a.w);
        }
      }
    }
  }
}

}  // namespace vfd

// ================================================================================== C ABI
using namespace vfd;

static int check_voxel_desc(const vfd_voxel_desc* d) {
  VFD_REQUIRE(d != nullptr, "null descriptor");
  VFD_REQUIRE(d->B > 0 && d->N > 0 && d->N <= 8, "bad B/N (%d, %d)", d->B, d->N);
  VFD_REQUIRE(d->h > 1 && d->w > 1 && d->X > 1 && d->Y > 1 && d->Z > 1, "bad map / voxel sizes");
  VFD_REQUIRE(d->axis_x && d->axis_y && d->axis_z, "voxel axes not set");
  return VFD_OK;
}

extern "C" {

int vfd_mask_downsample(const vfd_voxel_desc* d, const float* mask, float* mask_lo, void* stream) {
  int st = check_voxel_desc(d);
  if (st) return st;
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_MASK_DOWN, s);
  const int n = d->B * d->N * d->h * d->w;
  mask_downsample_k<<<cdiv(n, 256), 256, 0, s>>>(mask, mask_lo, d->B * d->N, d->H, d->W, d->h, d->w);
  return fail_launch("mask_downsample");
}

int vfd_fuse_depth_fwd(const vfd_voxel_desc* d, const float* P, const float* mask_lo, const float* K,
                       const float* Einv, const float* wz, const float* b_no, const float* b_o,
                       float* vox, void* stream) {
  int st = check_voxel_desc(d);
  if (st) return st;
  VFD_REQUIRE(d->Cv > 0 && d->Cv <= 128, "Cv=%d unsupported (<=128)", d->Cv);
  VFD_REQUIRE(d->group != nullptr, "camera groups not set");
  hipStream_t s = (hipStream_t)stream;
  const int V = d->X * d->Y * d->Z;
  dim3 grid(cdiv(cdiv(V, 64), 4), d->B);
  ProfScope ps(K_FUSE_DEPTH_FWD, s);
  const bool al = ((uintptr_t)P & 15) == 0 && ((uintptr_t)vox & 15) == 0 && ((uintptr_t)wz & 15) == 0 &&
                  ((uintptr_t)b_no & 15) == 0 && ((uintptr_t)b_o & 15) == 0;
  if (al && d->Cv == 64)
    fuse_depth_fwd_q_k<64><<<grid, 256, 0, s>>>(*d, P, mask_lo, K, Einv, wz, b_no, b_o, vox);
  else if (al && d->Cv == 32)
    fuse_depth_fwd_q_k<32><<<grid, 256, 0, s>>>(*d, P, mask_lo, K, Einv, wz, b_no, b_o, vox);
  else if (al && d->Cv == 16)
    fuse_depth_fwd_q_k<16><<<grid, 256, 0, s>>>(*d, P, mask_lo, K, Einv, wz, b_no, b_o, vox);
  else if (d->Cv <= 64)
    fuse_depth_fwd_k<1><<<grid, 256, 0, s>>>(*d, P, mask_lo, K, Einv, wz, b_no, b_o, vox);
  else
    fuse_depth_fwd_k<2><<<grid, 256, 0, s>>>(*d, P, mask_lo, K, Einv, wz, b_no, b_o, vox);
  return fail_launch("fuse_depth_fwd");
}

size_t vfd_fuse_depth_bwd_workspace(const vfd_voxel_desc* d) {
  const int V = d->X * d->Y * d->Z;
  return (size_t)d->B * cdiv(V, 64) * 5 * d->Cv * sizeof(float);
}

int vfd_fuse_depth_bwd(const vfd_voxel_desc* d, const float* d_vox, const float* vox, const float* mask_lo,
                       const float* K, const float* Einv, float* dP, float* d_wzb, void* ws, size_t ws_bytes,
                       void* stream) {
  int st = check_voxel_desc(d);
  if (st) return st;
  VFD_REQUIRE(d->Cv > 0 && d->Cv <= 128, "Cv=%d unsupported (<=128)", d->Cv);
  VFD_REQUIRE(ws_bytes >= vfd_fuse_depth_bwd_workspace(d), "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int V = d->X * d->Y * d->Z;
  ProfScope ps(K_FUSE_DEPTH_BWD, s);         // the op: zero dP, scatter, partial reduction
  zero_async(dP, (size_t)d->B * d->N * d->h * d->w * 2 * d->Cv * sizeof(float), s);
  dim3 grid(cdiv(cdiv(V, 64), 4), d->B);
  float* partial = (float*)ws;
  if (d->Cv <= 64)
    fuse_depth_bwd_k<1, true><<<grid, 256, 0, s>>>(*d, d_vox, vox, mask_lo, K, Einv, dP, partial);
  else
    fuse_depth_bwd_k<2, true><<<grid, 256, 0, s>>>(*d, d_vox, vox, mask_lo, K, Einv, dP, partial);
  st = fail_launch("fuse_depth_bwd");
  if (st) return st;
  // pad waves beyond V wrote nothing: zero-initialise by reducing only real rows
  const int rows = d->B * (int)cdiv(V, 64);
  fuse_depth_reduce_k<<<5 * d->Cv, 256, 0, s>>>(partial, rows, 5 * d->Cv, d_wzb);
  return fail_launch("fuse_depth_reduce");
}

// plan buffer: [B*N][V] PlanEntry | [B*N][hw+1] int row_ptr | [B*N][4V] int csr
static size_t plan_entries_bytes(const vfd_voxel_desc* d) {
  return (size_t)d->B * d->N * d->X * d->Y * d->Z * sizeof(PlanEntry);
}
static int host_tiles(const vfd_voxel_desc* d) { return cdiv(d->w, PT) * cdiv(d->h, PT); }
static size_t plan_rowptr_bytes(const vfd_voxel_desc* d) {
  return ((size_t)d->B * d->N * (host_tiles(d) * PSUB + 1) * sizeof(int) + 255) / 256 * 256;
}
static size_t plan_cursor_bytes(const vfd_voxel_desc* d) {
  return ((size_t)d->B * d->N * host_tiles(d) * PSUB * sizeof(int) + 255) / 256 * 256;
}

static size_t plan_items_bytes(const vfd_voxel_desc* d) {
  return (size_t)d->B * d->N * 4 * d->X * d->Y * d->Z * sizeof(TileItem);
}
static size_t plan_tasks_bytes(const vfd_voxel_desc* d) {     // independent of C (see plan_task_k)
  return ((size_t)(d->B * d->N * host_tiles(d) + PBW_POOL + PBW_POOL / 2) * sizeof(int4) + 255) / 256 * 256;
}

static size_t plan_fold_bytes(const vfd_voxel_desc* d) {       // K2 backward's folded border rows
  return ((size_t)d->B * 2 * (d->X + d->Y) * d->Z * (POSE_MAXC + 1) * sizeof(float) + 255) / 256 * 256;
}

static constexpr size_t PLAN_POOL_BYTES = (size_t)PBW_POOL * PT2 * POSE_MAXC * sizeof(float);

size_t vfd_fusion_plan_bytes(const vfd_voxel_desc* d) {
  // deterministic mode: + an item array for the bucket ordering pass
  return plan_entries_bytes(d) + plan_rowptr_bytes(d) + plan_cursor_bytes(d) + plan_items_bytes(d) +
         plan_tasks_bytes(d) + 256 + plan_fold_bytes(d) + PLAN_POOL_BYTES +
         (d->deterministic ? plan_items_bytes(d) : 0);
}

int vfd_fusion_plan(const vfd_voxel_desc* d, const float* mask_lo, const float* K, const float* Einv, void* plan,
                    int* counts, void* stream) {
  int st = check_voxel_desc(d);
  if (st) return st;
  VFD_REQUIRE((size_t)d->X * d->Y * d->Z < (1u << 24), "voxel grid too large for the plan (%d x %d x %d)", d->X, d->Y, d->Z);
  VFD_REQUIRE((size_t)(d->X + 2) * (d->Y + 2) < (1u << 20) && d->Z < 256, "voxel grid too large for the pose index");
  VFD_REQUIRE(2 * (size_t)host_tiles(d) * PSUB * sizeof(int) <= 160 * 1024, "feature map %dx%d too large for the tile index", d->h, d->w);
  hipStream_t s = (hipStream_t)stream;
  const int V = d->X * d->Y * d->Z;
  zero_async(counts, (size_t)d->B * d->N * sizeof(int), s);
  dim3 grid(cdiv(V, 256), d->B);
  ProfScope ps(K_FUSION_PLAN, s);
  switch (d->N) {
#define VFD_CASE(n) case n: fusion_plan_k<n><<<grid, 256, 0, s>>>(*d, mask_lo, K, Einv, (PlanEntry*)plan, counts); break;
    VFD_CASE(1) VFD_CASE(2) VFD_CASE(3) VFD_CASE(4) VFD_CASE(5) VFD_CASE(6) VFD_CASE(7) VFD_CASE(8)
#undef VFD_CASE
  }
  int* row_ptr = (int*)((char*)plan + plan_entries_bytes(d));
  int* cursor = (int*)((char*)row_ptr + plan_rowptr_bytes(d));
  TileItem* csr = (TileItem*)((char*)cursor + plan_cursor_bytes(d));
  zero_async(cursor, (size_t)d->B * d->N * host_tiles(d) * PSUB * sizeof(int), s);
  const dim3 egrid(cdiv(V, 256), d->B * d->N);
  const size_t hist = (size_t)host_tiles(d) * PSUB * sizeof(int);
  if (2 * hist > 64 * 1024) {
    (void)hipFuncSetAttribute((const void*)plan_count_k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)hist);
    (void)hipFuncSetAttribute((const void*)plan_fill_k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(2 * hist));
  }
  plan_count_k<<<egrid, 256, hist, s>>>(*d, (const PlanEntry*)plan, counts, cursor);
  plan_scan_k<<<d->B * d->N, PIDX_THREADS, 0, s>>>(*d, cursor, row_ptr);
  plan_fill_k<<<egrid, 256, 2 * hist, s>>>(*d, (const PlanEntry*)plan, counts, cursor, csr);
  if (d->deterministic) {
    TileItem* tmp = (TileItem*)((char*)plan + vfd_fusion_plan_bytes(d) - plan_items_bytes(d));
    const dim3 igrid(cdiv(4 * V, 256), d->B * d->N);
    plan_order_k<<<igrid, 256, 0, s>>>(*d, row_ptr, csr, tmp);
    plan_copy_k<<<igrid, 256, 0, s>>>(*d, row_ptr, tmp, csr);
  }
  int4* tasks = (int4*)((char*)csr + plan_items_bytes(d));
  int* ctrl = (int*)((char*)tasks + plan_tasks_bytes(d));
  int4* combos = tasks + (d->B * d->N * host_tiles(d) + PBW_POOL);
  plan_task_k<<<1, 1024, 0, s>>>(*d, row_ptr, tasks, combos, ctrl);
  return fail_launch("fusion_plan");
}

int vfd_fuse_pose_fwd_t(const vfd_voxel_desc* d, const float* mask_lo, const float* K, const float* Einv,
                        const float* feats_cl, void* out, int dtype_out, const int* order, int order_cap,
                        void* stream) {
  int st = check_voxel_desc(d);
  if (st) return st;
  VFD_REQUIRE(d->C >= 1 && d->C <= POSE_MAXC, "fuse_pose: C=%d outside [1, %d]", d->C, POSE_MAXC);
  VFD_REQUIRE(d->N >= 1 && d->N <= 8, "fuse_pose: N=%d outside [1, 8]", d->N);
  VFD_REQUIRE(dtype_out == 0 || dtype_out == 1, "fuse_pose: dtype_out %d (0 fp32, 1 bf16)", dtype_out);
  hipStream_t s = (hipStream_t)stream;
  const int V = d->X * d->Y * d->Z;
  VFD_REQUIRE(!order || (order_cap > 0 && 8 * (long long)order_cap >= V),
              "fuse_pose: order holds 8 x %d slots for %d voxels", order_cap, V);
  dim3 grid(order ? 8 * cdiv(order_cap, POSE_TV) : cdiv(V, POSE_TV), d->B);
  ProfScope ps(K_FUSE_POSE_FWD, s);
  switch (d->N * 2 + dtype_out) {
#define VFD_CASE(n)                                                                                               \
  case 2 * n: fuse_pose_fwd_k<n, float><<<grid, 256, 0, s>>>(*d, mask_lo, K, Einv, feats_cl, order, order_cap,    \
                                                             (float*)out); break;                                 \
  case 2 * n + 1: fuse_pose_fwd_k<n, __bf16><<<grid, 256, 0, s>>>(*d, mask_lo, K, Einv, feats_cl, order, order_cap, \
                                                                  (__bf16*)out); break;
    VFD_CASE(1) VFD_CASE(2) VFD_CASE(3) VFD_CASE(4) VFD_CASE(5) VFD_CASE(6) VFD_CASE(7) VFD_CASE(8)
#undef VFD_CASE
  }
  return fail_launch("fuse_pose_fwd");
}

int vfd_fuse_pose_fwd(const vfd_voxel_desc* d, const float* mask_lo, const float* K, const float* Einv,
                      const float* feats_cl, float* out, void* stream) {
  return vfd_fuse_pose_fwd_t(d, mask_lo, K, Einv, feats_cl, out, 0, nullptr, 0, stream);
}

// d_out of dtype_out (0 fp32, 1 bf16: the bf16 K2C data gradient)
int vfd_fuse_pose_bwd_t(const vfd_voxel_desc* d, const void* plan, const int* counts, const void* d_out, int dtype_out,
                        float* d_feats, void* stream) {
  int st = check_voxel_desc(d);
  if (st) return st;
  (void)counts;
  VFD_REQUIRE(d->C >= 4 && d->C <= POSE_MAXC && d->C % 4 == 0, "fuse_pose_bwd: C=%d must be a multiple of 4 in [4, %d]", d->C, POSE_MAXC);
  VFD_REQUIRE(dtype_out == 0 || dtype_out == 1, "fuse_pose_bwd: dtype_out %d (0 fp32, 1 bf16)", dtype_out);
  hipStream_t s = (hipStream_t)stream;
  const int hw = d->h * d->w;
  const int* row_ptr = (const int*)((const char*)plan + plan_entries_bytes(d));
  const TileItem* csr = (const TileItem*)((const char*)row_ptr + plan_rowptr_bytes(d) + plan_cursor_bytes(d));
  const int4* tasks = (const int4*)((const char*)csr + plan_items_bytes(d));
  const int* ctrl = (const int*)((const char*)tasks + plan_tasks_bytes(d));   // {tasks, split tiles}
  const int4* combos = tasks + (d->B * d->N * host_tiles(d) + PBW_POOL);
  float* fbuf = (float*)((char*)ctrl + 256);                   // folded border rows (plan scratch)
  float* pool = (float*)((char*)fbuf + plan_fold_bytes(d));    // split tiles' partials
  ProfScope ps(K_FUSE_POSE_BWD, s);
  const unsigned nfold = d->B * 2 * (d->X + d->Y) * POSE_FOLD_SPLIT;
  const int al16 = (((uintptr_t)d_out | (uintptr_t)fbuf) & 15) == 0;
  const int ntask_max = host_tiles(d) * d->B * d->N + PBW_POOL;
  const unsigned ntask = 128 * cdiv(ntask_max, 128);
  if (dtype_out == 1) {
    if (d->pad_out) pose_fold_k<__bf16><<<nfold, 256, 0, s>>>(*d, (const __bf16*)d_out, fbuf, al16);
    fuse_pose_bwd_k<__bf16><<<ntask, 64, 0, s>>>(*d, tasks, ctrl, csr, (const __bf16*)d_out, fbuf, pool, d_feats);
  } else {
    if (d->pad_out) pose_fold_k<float><<<nfold, 256, 0, s>>>(*d, (const float*)d_out, fbuf, al16);
    fuse_pose_bwd_k<float><<<ntask, 64, 0, s>>>(*d, tasks, ctrl, csr, (const float*)d_out, fbuf, pool, d_feats);
  }
  pose_combine_k<<<std::min(PBW_POOL / 2, host_tiles(d) * d->B * d->N), PCB_THREADS, 0, s>>>(*d, combos, ctrl, pool, d_feats);
  return fail_launch("fuse_pose_bwd");
}

int vfd_fuse_pose_bwd(const vfd_voxel_desc* d, const void* plan, const int* counts, const float* d_out,
                      float* d_feats, void* stream) {
  return vfd_fuse_pose_bwd_t(d, plan, counts, d_out, 0, d_feats, stream);
}

// The planned K1 backward's split-tile partials live in ITS workspace, after the depth-column
// partials — not in the plan's pool, which the K2 backward of the same step uses: with the pose
// branch on its own stream the two backwards run concurrently, and a shared pool let each overwrite
// the other's partial tiles (round 6: wrong d feats for both in HIP-graph replays, where the two
// overlap most; tests/graph_det_worker.py).
static size_t k1_partial_bytes(const vfd_voxel_desc* d) {
  return (vfd_fuse_depth_bwd_workspace(d) + 255) / 256 * 256;
}

size_t vfd_fuse_depth_bwd_planned_workspace(const vfd_voxel_desc* d) {
  return k1_partial_bytes(d) + PLAN_POOL_BYTES;
}

int vfd_fuse_depth_bwd_planned(const vfd_voxel_desc* d, const void* plan, const float* d_vox, const float* vox,
                               const float* mask_lo, const float* K, const float* Einv, float* dP, float* d_wzb,
                               void* ws, size_t ws_bytes, void* stream) {
  int st = check_voxel_desc(d);
  if (st) return st;
  VFD_REQUIRE(d->Cv == K1G_CV, "fuse_depth_bwd_planned: Cv=%d (the gather backward needs %d)", d->Cv, K1G_CV);
  VFD_REQUIRE(plan && d_vox && vox && dP && d_wzb && ws, "fuse_depth_bwd_planned: null argument");
  VFD_REQUIRE(ws_bytes >= vfd_fuse_depth_bwd_planned_workspace(d),
              "fuse_depth_bwd_planned: workspace too small (vfd_fuse_depth_bwd_planned_workspace)");
  hipStream_t s = (hipStream_t)stream;
  const int V = d->X * d->Y * d->Z;
  const int* row_ptr = (const int*)((const char*)plan + plan_entries_bytes(d));
  const TileItem* csr = (const TileItem*)((const char*)row_ptr + plan_rowptr_bytes(d) + plan_cursor_bytes(d));
  const int4* tasks = (const int4*)((const char*)csr + plan_items_bytes(d));
  const int* ctrl = (const int*)((const char*)tasks + plan_tasks_bytes(d));
  const int4* combos = tasks + (d->B * d->N * host_tiles(d) + PBW_POOL);
  float* pool = (float*)((char*)ws + k1_partial_bytes(d));      // this call's own split-tile partials
  ProfScope ps(K_FUSE_DEPTH_BWD, s);
  const int ntask_max = host_tiles(d) * d->B * d->N + PBW_POOL;
  fuse_depth_bwd_gather_k<<<128 * cdiv(ntask_max, 128), 64, 0, s>>>(*d, tasks, ctrl, csr, d_vox, vox, pool, dP);
  fuse_depth_combine_k<<<std::min(PBW_POOL / 2, host_tiles(d) * d->B * d->N), K1C_THREADS, 0, s>>>(
      *d, combos, ctrl, pool, dP);
  // depth-column and bias gradients: the voxel walk without the scatter
  dim3 grid(cdiv(cdiv(V, 64), 4), d->B);
  float* partial = (float*)ws;
  fuse_depth_bwd_k<1, false><<<grid, 256, 0, s>>>(*d, d_vox, vox, mask_lo, K, Einv, dP, partial);
  st = fail_launch("fuse_depth_bwd_planned");
  if (st) return st;
  const int rows = d->B * (int)cdiv(V, 64);
  fuse_depth_reduce_k<<<5 * d->Cv, 256, 0, s>>>(partial, rows, 5 * d->Cv, d_wzb);
  return fail_launch("fuse_depth_reduce");
}

int vfd_voxel_project_fwd(const vfd_voxel_desc* d, const float* vox, const float* invK, const float* E,
                          float* out, void* stream) {
  int st = check_voxel_desc(d);
  if (st) return st;
  VFD_REQUIRE(d->dbins != nullptr && d->D > 0, "depth bins not set");
  hipStream_t s = (hipStream_t)stream;
  VFD_REQUIRE(d->Cv <= 64, "voxel_project: Cv=%d > 64", d->Cv);
  VFD_REQUIRE(((uintptr_t)vox & 15) == 0 && ((uintptr_t)out & 15) == 0, "voxel_project: 16-B aligned buffers required");
  const int ntask = cdiv((size_t)d->h * d->w * d->D, VP_S) * d->B * d->N;
  dim3 grid(8 * cdiv(ntask, 8));
  ProfScope ps(K_VPROJ_FWD, s);
  switch (d->Cv) {
    case 8: voxel_project_fwd_k<8><<<grid, 256, 0, s>>>(*d, vox, invK, E, out); break;
    case 16: voxel_project_fwd_k<16><<<grid, 256, 0, s>>>(*d, vox, invK, E, out); break;
    case 32: voxel_project_fwd_k<32><<<grid, 256, 0, s>>>(*d, vox, invK, E, out); break;
    case 64: voxel_project_fwd_k<64><<<grid, 256, 0, s>>>(*d, vox, invK, E, out); break;
    default: set_error("voxel_project: Cv=%d unsupported (8/16/32/64)", d->Cv); return VFD_EINVAL;
  }
  return fail_launch("voxel_project_fwd");
}

#ifndef VFD_VPB_WORKERS
#define VFD_VPB_WORKERS 5120
#endif
constexpr int VPB_WORKERS = VFD_VPB_WORKERS;      // persistent waves (20 per CU: LDS 8.4 KB, <=96 VGPRs)

struct VpbWs {
  size_t cnt, zero, ptr, bsum, boff, rank, entries, fold, parts, tasks, ctrl, total;
};
static VpbWs vpb_ws(const vfd_voxel_desc* d) {
  const VpbGeom g = vpb_geom(*d);
  const size_t ncell = (size_t)d->B * g.ncell, nS = (size_t)d->B * d->N * d->h * d->w * d->D;
  const size_t nblk = cdiv(ncell, VB_SCAN), nb = (size_t)d->B * g.ntile;
  const size_t ntask_max = nb + cdiv(8 * nS, VB_S);
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  VpbWs w;
  w.cnt = 0;
  w.zero = al(ncell * 4);              // one zero row of 64 floats right after the counters,
  w.fold = w.zero + (size_t)d->Cv * 4;  // then the folded rows (fbz = zero row + fold rows)
  w.ptr = al(w.fold + (size_t)d->B * d->N * 2 * (d->w + d->h) * d->D * d->Cv * 4);
  w.bsum = w.ptr + al(ncell * 4);
  w.boff = w.bsum + al(nblk * 4);
  w.rank = w.boff + al((nblk + 1) * 4);
  w.entries = w.rank + al(nS * 4);
  w.parts = w.entries + al(nS * 16);
  w.tasks = w.parts + al(nb * 4);
  w.ctrl = w.tasks + al(ntask_max * 8);
  w.total = w.ctrl + al(16 * 4);
  return w;
}

// The geometry-only half of the backward (the counting sort of the frustum samples by voxel cell,
// the tile parts and the task list) depends on invK / E / the depth bins, not on d_out: it is its
// own call so the caller can build it while the forward's dense layers run (side stream).
static int vpb_check(const vfd_voxel_desc* d) {
  int st = check_voxel_desc(d);
  if (st) return st;
  VFD_REQUIRE(d->dbins != nullptr && d->D > 0, "depth bins not set");
  VFD_REQUIRE(d->Cv == 8 || d->Cv == 16 || d->Cv == 32 || d->Cv == 64, "voxel_project: Cv=%d unsupported (8/16/32/64)", d->Cv);
  VFD_REQUIRE((size_t)d->B * d->N * d->h * d->w * d->D < (1u << 31) / 2, "voxel_project_bwd: too many samples");
  const size_t dout_rows = (size_t)d->B * d->N * (d->h + 2 * (d->pad_out ? 1 : 0)) * (d->w + 2 * (d->pad_out ? 1 : 0)) * d->D;
  VFD_REQUIRE(dout_rows < (1ull << 31), "voxel_project_bwd: d_out has too many rows for 31-bit row indices");
  return VFD_OK;
}

struct VpbPtrs {
  int *cnt, *ptr, *bsum, *boff, *rank, *parts, *ctrl;
  float4* entries;
  float* fb;
  const float* zrow;
  int2* tasks;
};

static VpbPtrs vpb_ptrs(const VpbWs& w, void* ws) {
  char* base = (char*)ws;
  VpbPtrs p;
  p.cnt = (int*)(base + w.cnt);
  p.ptr = (int*)(base + w.ptr);
  p.bsum = (int*)(base + w.bsum);
  p.boff = (int*)(base + w.boff);
  p.rank = (int*)(base + w.rank);
  p.entries = (float4*)(base + w.entries);
  p.fb = (float*)(base + w.fold);
  p.zrow = (const float*)(base + w.zero);
  p.parts = (int*)(base + w.parts);
  p.tasks = (int2*)(base + w.tasks);
  p.ctrl = (int*)(base + w.ctrl);
  return p;
}

static void vpb_plan_launch(const vfd_voxel_desc* d, const float* invK, const float* E, void* ws, hipStream_t s) {
  const VpbWs w = vpb_ws(d);
  const VpbGeom g = vpb_geom(*d);
  const VpbPtrs p = vpb_ptrs(w, ws);
  const int ncell = d->B * g.ncell, nblk = cdiv(ncell, VB_SCAN), nb = d->B * g.ntile;
  const int hwD = d->h * d->w * d->D;
  zero_async(p.cnt, w.fold, s);   // counters + zero row
  const int cpb = cdiv(hwD, 256);
  vpb_count_k<<<cpb * d->B * d->N, 256, 0, s>>>(*d, invK, E, p.cnt, p.rank, cpb);
  vpb_scan1_k<<<nblk, 256, 0, s>>>(p.cnt, ncell, p.ptr, p.bsum);
  vpb_scan2_k<<<1, 1024, 0, s>>>(p.bsum, nblk, p.boff);
  vpb_fill_k<<<dim3(cpb, d->B * d->N), 256, 0, s>>>(*d, invK, E, p.rank, p.ptr, p.boff, p.entries);
  if (d->deterministic) {
    vpb_order_k<<<cdiv((size_t)d->B * d->N * hwD, 256), 256, 0, s>>>(*d, p.ptr, p.boff, p.entries, p.rank);
    vpb_fill_k<<<dim3(cpb, d->B * d->N), 256, 0, s>>>(*d, invK, E, p.rank, p.ptr, p.boff, p.entries);
  }
  vpb_tile_k<<<nb, 64, 0, s>>>(*d, p.ptr, p.boff, p.parts);
  vpb_tasks_k<<<1, 1024, 0, s>>>(p.parts, nb, p.tasks, p.ctrl);
}

static void vpb_bwd_launch(const vfd_voxel_desc* d, const float* d_out, void* ws, float* d_vox, hipStream_t s) {
  const VpbWs w = vpb_ws(d);
  const VpbGeom g = vpb_geom(*d);
  const VpbPtrs p = vpb_ptrs(w, ws);
  const int nb = d->B * g.ntile;
  const int nf = d->pad_out == 1 ? d->B * d->N * 2 * (d->w + d->h) : 0;
  switch (d->Cv) {
#define VPB_LAUNCH(CVV)                                                                                         \
  case CVV:                                                                                                     \
    vpb_fold_zero_k<CVV><<<nf + nb + 1, 256, 0, s>>>(*d, d_out, p.fb, nf, p.parts, nb, p.ctrl, d_vox);            \
    vpb_main_k<CVV><<<VPB_WORKERS / VB_LG, 64 * VB_LG, 0, s>>>(*d, p.ptr, p.boff, p.entries, p.tasks, p.ctrl, d_out, \
                                                                 p.zrow, d_vox);                                \
    break;
    VPB_LAUNCH(8)
    VPB_LAUNCH(16)
    VPB_LAUNCH(32)
    VPB_LAUNCH(64)
#undef VPB_LAUNCH
  }
}

size_t vfd_voxel_project_plan_bytes(const vfd_voxel_desc* d) {
  if (vpb_check(d)) return 0;
  return vpb_ws(d).total;
}

size_t vfd_voxel_project_bwd_workspace(const vfd_voxel_desc* d) { return vfd_voxel_project_plan_bytes(d); }

int vfd_voxel_project_plan(const vfd_voxel_desc* d, const float* invK, const float* E, void* plan,
                           size_t plan_bytes, void* stream) {
  int st = vpb_check(d);
  if (st) return st;
  VFD_REQUIRE(plan != nullptr && plan_bytes >= vpb_ws(d).total, "voxel_project_plan: buffer %zu < %zu bytes",
              plan_bytes, vpb_ws(d).total);
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_VPROJ_PLAN, s);
  vpb_plan_launch(d, invK, E, plan, s);
  return fail_launch("voxel_project_plan");
}

int vfd_voxel_project_bwd_planned(const vfd_voxel_desc* d, const float* d_out, void* plan, size_t plan_bytes,
                                  float* d_vox, void* stream) {
  int st = vpb_check(d);
  if (st) return st;
  VFD_REQUIRE(((uintptr_t)d_vox & 15) == 0, "voxel_project: 16-B aligned d_vox required");
  VFD_REQUIRE(plan != nullptr && plan_bytes >= vpb_ws(d).total, "voxel_project_bwd: plan %zu < %zu bytes",
              plan_bytes, vpb_ws(d).total);
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_VPROJ_BWD, s);
  vpb_bwd_launch(d, d_out, plan, d_vox, s);
  return fail_launch("voxel_project_bwd");
}

int vfd_voxel_project_bwd(const vfd_voxel_desc* d, const float* d_out, const float* invK, const float* E,
                          float* d_vox, void* ws, size_t ws_bytes, void* stream) {
  int st = vpb_check(d);
  if (st) return st;
  VFD_REQUIRE(((uintptr_t)d_vox & 15) == 0, "voxel_project: 16-B aligned d_vox required");
  VFD_REQUIRE(ws != nullptr && ws_bytes >= vpb_ws(d).total, "voxel_project_bwd: workspace %zu < %zu bytes", ws_bytes,
              vpb_ws(d).total);
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_VPROJ_BWD, s);
  vpb_plan_launch(d, invK, E, ws, s);
  vpb_bwd_launch(d, d_out, ws, d_vox, s);
  return fail_launch("voxel_project_bwd");
}

}  // extern "C"
