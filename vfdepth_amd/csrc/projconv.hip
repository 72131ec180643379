// K3C — voxel -> frustum trilinear resampling FUSED into reduce_dim's first 3x3 conv, as an
// fp32 MFMA implicit GEMM (network/volumetric_fusionnet.py:59-60, 232-267, depth mode).
//
// The reference materialises, per camera, the frustum features X[Cv*D, h, w] (trilinear samples of
// the voxel grid on D depth planes) and convolves them (3x3, reflect padding, Cv*D -> O = 256)
// followed by LeakyReLU(0.1).  Here X is never written to HBM:
//
//   Y[n, y, x, o] = lrelu(bias[o] + sum_{d, c, ky, kx} W[o, c*D + d, ky, kx] * Xp[n, y+ky, x+kx, d, c])
//
// is an implicit GEMM with M = pixels (B*N*h*w), N = O output channels, K = D * Cv * 9, whose
// A operand (pixels x k) is generated on the fly: for one (pixel tile, depth bin d) "atom" the
// workgroup gathers the Cv-channel trilinear samples of the tile's reflect-padded halo into LDS
// (8 voxel rows per sample from the channels-last [B, V, Cv] grid, the K3 arithmetic exactly), then
// runs the 9 taps x Cv channels of that depth bin on v_mfma_f32_32x32x2_f32 (exact fp32 FMA chains:
// the reference's fp32 conv up to summation order).  B operands (weights) are read straight from
// L2 / Infinity Cache in a fragment-ordered copy of W (`vfd_proj_conv_weight_layout`).
//
// Work split ("stream-K"): the B*N * tiles * D atoms, tile-major, are cut into equal contiguous
// ranges, one per workgroup (one resident per CU): a range covers at most two tiles, whose partial
// sums go to a per-(workgroup, slot) buffer in MFMA fragment order; `pcv_reduce_k` sums each tile's
// partials in workgroup order (deterministic), adds the bias, applies the LeakyReLU and writes the
// reflect-padded NHWC input of reduce_dim's second conv.
#include <type_traits>

#include "vfd_common.h"

namespace vfd {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int PC_CV = 64;                       // voxel channels (voxel_pre_dim[-1])
constexpr int PC_O = 256;                       // output channels (reduce_dim[0])
constexpr int PC_TR = 8, PC_TC = 16;            // pixel tile: 8 rows x 16 columns = 128 pixels
constexpr int PC_PIX = PC_TR * PC_TC;
constexpr int PC_HR = PC_TR + 2, PC_HC = PC_TC + 2;
constexpr int PC_NPOS = PC_HR * PC_HC;          // 180 halo positions
constexpr int PC_XS = PC_CV + 4;                // LDS floats per halo position (16-B aligned rows)
constexpr int PC_WAVES = 4;                     // each wave: 128 pixels x 64 output channels
constexpr int PC_FRAG = PC_PIX * PC_O;          // floats of one tile's partial (fragment order)
constexpr int PC_WG_PER_CU = 1;

struct PcGeom {
  int tr, tc, tiles_img, ntile, natom, ngroup;
};

__host__ __device__ inline PcGeom pc_geom(const vfd_voxel_desc& d, int ngroup) {
  PcGeom g;
  g.tr = (d.h + PC_TR - 1) / PC_TR;
  g.tc = (d.w + PC_TC - 1) / PC_TC;
  g.tiles_img = g.tr * g.tc;
  g.ntile = d.B * d.N * g.tiles_img;
  g.natom = g.ntile * d.D;
  g.ngroup = ngroup;
  return g;
}

// first atom of workgroup g (ranges are [lo(g), lo(g+1)))
__host__ __device__ inline int pc_lo(const PcGeom& g, int grp) {
  return (int)(((long long)grp * g.natom) / g.ngroup);
}

__device__ __forceinline__ int pc_reflect(int i, int n) {
  // reflect-pad(1) source row of padded-relative index i in [-1, n]; rows of a partial tile that
  // lie beyond the image are clamped (their outputs are never stored)
  if (i < 0) return 1 < n ? 1 : 0;
  if (i >= n) return i == n ? (n >= 2 ? n - 2 : 0) : n - 1;
  return i;
}

// Workgroup = 8 waves, one per CU: waves 0-3 are the MFMA "compute" waves (each 128 pixels x 64
// output channels, 8 f32x16 accumulators), waves 4-7 the "gather" waves, which build the NEXT
// atom's halo samples into the other half of a double-buffered LDS image while the compute waves
// run the current one (one barrier per atom).  Compute waves therefore never stall on the voxel
// gather; each keeps its SIMD's matrix pipe busy alone, with the weight fragments prefetched
// PC_PF iterations ahead from L2 / Infinity Cache.
constexpr int PC_THREADS = 512;
#ifndef VFD_PC_PF
#define VFD_PC_PF 4
#endif
constexpr int PC_PF = VFD_PC_PF;                // weight-fragment prefetch distance (iterations)
constexpr int PC_ITERS = 9 * (PC_CV / 4);       // (tap, channel quad) iterations per atom

// gather waves: halo samples of atom (tile origin y0/x0, depth bin di) into one LDS image, and —
// when `xo` is given — the tile's own (interior) samples into the padded NHWC frustum-feature map
// the conv's backward reads (K3's output layout; written once, reflect copies included).
constexpr int PC_GPOS = (PC_NPOS + 15) / 16 * 4;   // halo positions per gather wave (48)
#ifndef VFD_PH_PIPE
#define VFD_PH_PIPE 0                               // bf16 K3C dgrad loader two atoms ahead: 965 vs 932 us, off
#endif
#ifndef VFD_PCVB_XO_COMPUTE
#define VFD_PCVB_XO_COMPUTE 1                       // bf16 K3C: side output written by the compute waves
#endif
#ifndef VFD_PCG_U
#define VFD_PCG_U 4                                 // gather: positions' corner rows in flight per lane
#endif

struct PcTri {
  int base;
  unsigned in;
  float w[8];
};

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// one (position, channel quad) sample into a row of T: fp32 (float4, 16 B) or bf16 (8 B, the
// fp32 trilinear sum rounded to nearest even, as torch's .to(bfloat16) of K3's fp32 output)
__device__ __forceinline__ void pc_put(float* dst, float4 v) { *reinterpret_cast<float4*>(dst) = v; }
__device__ __forceinline__ void pc_put(__bf16* dst, float4 v) {
  bf16x4 b;
  b[0] = (__bf16)v.x;
  b[1] = (__bf16)v.y;
  b[2] = (__bf16)v.z;
  b[3] = (__bf16)v.w;
  *reinterpret_cast<bf16x4*>(dst) = b;
}

template <typename T, int XS>
__device__ __forceinline__ void pc_gather(const vfd_voxel_desc& d, T* __restrict__ xs, PcTri* __restrict__ tw,
                                          const float* __restrict__ vox_b, const float* __restrict__ iK,
                                          const float* __restrict__ E, int y0, int x0, int di, int gw,
                                          T* __restrict__ xo) {
  const int lane = threadIdx.x & 63;
  // (1) the wave's positions p = gw*4 + (k & 3) + 16*(k >> 2): lane k evaluates slot k's trilinear
  //     cell once (wave-private LDS slice, no workgroup barrier)
  if (lane < PC_GPOS) {
    const int p = gw * 4 + (lane & 3) + 16 * (lane >> 2);
    if (p < PC_NPOS) {
      const int hr = p / PC_HC, hc = p - hr * PC_HC;
      const int py = pc_reflect(y0 + hr - 1, d.h), px = pc_reflect(x0 + hc - 1, d.w);
      const Tri t = frustum_sample(d, iK, E, px, py, d.dbins[di]);
      tw[lane].base = (t.z0 * d.Y + t.y0) * d.X + t.x0;
      tw[lane].in = t.in;
#pragma unroll
      for (int k = 0; k < 8; ++k) tw[lane].w[k] = t.w[k];
    }
  }
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
  // (2) lanes = (position, channel quad): 16 quads per 64-channel row, 4 positions per instruction;
  //     U positions' 8 corner rows in flight together (the voxel rows come from L2 / MALL at ~1 us:
  //     one position at a time made the bf16 kernel's gather, not its MFMAs, the bound)
  const int q = lane & 15, sub = lane >> 4;
  const float4* vb = reinterpret_cast<const float4*>(vox_b) + q;
  const int wo = d.w + 2;
  constexpr int U = VFD_PCG_U;
  static_assert((PC_GPOS / 4) % U == 0, "gather unroll");
  for (int i0 = 0; i0 < PC_GPOS / 4; i0 += U) {
    float4 v[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int it = i0 + u;
      const int p = gw * 4 + sub + 16 * it;
      const PcTri& t = tw[it * 4 + sub];
      const unsigned in = p < PC_NPOS ? t.in : 0u;
      const int base = t.base;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const bool ok = (in >> k & 1u) != 0u;
        v[u][k] = vb[(size_t)(ok ? base + corner_offset(d, k) : 0) * (PC_CV / 4)];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int it = i0 + u;
      const int p = gw * 4 + sub + 16 * it;
      if (p >= PC_NPOS) break;
      const PcTri& t = tw[it * 4 + sub];
      const unsigned in = t.in;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < 8; ++k) {           // K3's arithmetic: corner order, weight 0 when out of range
        const float w = (in >> k & 1u) ? t.w[k] : 0.f;
        acc.x += v[u][k].x * w;
        acc.y += v[u][k].y * w;
        acc.z += v[u][k].z * w;
        acc.w += v[u][k].w * w;
      }
      pc_put(&xs[p * XS + 4 * q], acc);
      if (xo) {
        const int hr = p / PC_HC, hc = p - hr * PC_HC;
        const int py = y0 + hr - 1, px = x0 + hc - 1;
        if (hr >= 1 && hr <= PC_TR && hc >= 1 && hc <= PC_TC && py < d.h && px < d.w) {
          int rows[3], cols[3], nr, nc;
          pad_sets(py, d.h, true, rows, &nr);
          pad_sets(px, d.w, true, cols, &nc);
          for (int r = 0; r < nr; ++r)
            for (int c = 0; c < nc; ++c) pc_put(xo + (((size_t)rows[r] * wo + cols[c]) * d.D + di) * PC_CV + 4 * q, acc);
        }
      }
    }
  }
}

struct PcAtom {
  int t, di, bc, y0, x0;
};

__device__ __forceinline__ PcAtom pc_atom(const vfd_voxel_desc& d, const PcGeom& g, int atom) {
  PcAtom a;
  a.t = atom / d.D;
  a.di = atom - a.t * d.D;
  a.bc = a.t / g.tiles_img;
  const int ti = a.t - a.bc * g.tiles_img;
  a.y0 = (ti / g.tc) * PC_TR;
  a.x0 = (ti % g.tc) * PC_TC;
  return a;
}

// Weight layout Wq (fragment order): [D][9 taps][Cv/4 = 16 quads][O][2 (h)][2 (s)], where the
// reference channel is c*D + d with c = 4*quad + 2*h + s.  For iteration i = tap*16 + quad of
// depth bin d, lane l of output block ob reads the float2 (s = 0, 1) at float2 index
// (d*144 + i)*2*O + (ob*32 + (l & 31))*2 + (l >> 5).
__global__ __launch_bounds__(PC_THREADS, 2) void pcv_main_k(vfd_voxel_desc d, PcGeom g,
                                                           const float* __restrict__ vox,
                                                           const float* __restrict__ invK,
                                                           const float* __restrict__ E,
                                                           const float* __restrict__ Wq,
                                                           float* __restrict__ partial,
                                                           float* __restrict__ xout) {
  __shared__ float xs[2][PC_NPOS * PC_XS];
  __shared__ PcTri tri[PC_WAVES][PC_GPOS];
  const int grp = blockIdx.x;
  const int a_lo = pc_lo(g, grp), a_hi = pc_lo(g, grp + 1);
  if (a_lo >= a_hi) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int V = d.X * d.Y * d.Z;
  const bool compute = wv < PC_WAVES;
  // prologue: the gather waves build the first atom
  auto gather = [&](int atom, float* dst) {
    const PcAtom a = pc_atom(d, g, atom);
    float* xo = xout ? xout + (size_t)a.bc * (d.h + 2) * (d.w + 2) * d.D * PC_CV : nullptr;
    pc_gather<float, PC_XS>(d, dst, tri[wv - PC_WAVES], vox + (size_t)(a.bc / d.N) * V * PC_CV, invK + a.bc * 16,
                            E + a.bc * 16, a.y0, a.x0, a.di, wv - PC_WAVES, xo);
  };
  if (!compute) gather(a_lo, xs[0]);
  __syncthreads();
  if (!compute) {
    // producer: atom a+1 into the other buffer while the compute waves run atom a
    for (int atom = a_lo; atom < a_hi; ++atom) {
      if (atom + 1 < a_hi)
        gather(atom + 1, xs[(atom + 1 - a_lo) & 1]);
      __syncthreads();
    }
    return;
  }
  const int li = lane & 31, lh = lane >> 5;
  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  // A-fragment LDS offsets of the wave's 4 pixel blocks at tap (0, 0), channel 2*lh
  int aoff[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int ip = 32 * a + li;                      // tile pixel of this lane's A row
    aoff[a] = ((ip >> 4) * PC_HC + (ip & 15)) * PC_XS + 2 * lh;
  }
  const float2* wlane = reinterpret_cast<const float2*>(Wq) + (size_t)(wv * 64 + li) * 2 + lh;
  // weight fragments of the flattened (atom, iteration) stream, PC_PF iterations ahead
  float2 bq[PC_PF][2];
  int pf_atom = a_lo, pf_it = 0;
  int pf_di = a_lo % d.D;                             // the prefetched atom's depth bin
  auto prefetch = [&](int slot) {
    if (pf_atom < a_hi) {
      const float2* w = wlane + ((size_t)pf_di * PC_ITERS + pf_it) * (2 * PC_O);
      bq[slot][0] = w[0];
      bq[slot][1] = w[64];
      if (++pf_it == PC_ITERS) {
        pf_it = 0;
        ++pf_atom;
        pf_di = pf_di + 1 == d.D ? 0 : pf_di + 1;
      }
    }
  };
#pragma unroll
  for (int k = 0; k < PC_PF; ++k) prefetch(k);
  int slot = 0;
  int tile = a_lo / d.D;
  for (int atom = a_lo; atom < a_hi; ++atom) {
    const int t = atom / d.D;
    if (t != tile) {                                  // flush the finished tile's partial
      float* dst = partial + ((size_t)grp * 2 + slot) * PC_FRAG + (size_t)wv * (PC_FRAG / PC_WAVES);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            dst[((a * 2 + b) * 16 + r) * 64 + lane] = acc[a][b][r];
            acc[a][b][r] = 0.f;
          }
      slot = 1;
      tile = t;
    }
    const float* xb = xs[(atom - a_lo) & 1];
    // A fragments software-pipelined one iteration ahead (LDS latency off the MFMA path)
    float2 afc[4], afn[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) afc[a] = *reinterpret_cast<const float2*>(&xb[aoff[a]]);
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap - 3 * ky;
      const float* xt = xb + (ky * PC_HC + kx) * PC_XS;
      const int tn = tap + 1, kyn = tn / 3, kxn = tn - 3 * kyn;
      const float* xn = xb + (kyn * PC_HC + kxn) * PC_XS;         // next tap (unused after tap 8)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ring = q % PC_PF;                   // 16 % PC_PF == 0: static ring slots
        const float2 b0 = bq[ring][0], b1 = bq[ring][1];
        prefetch(ring);
        if (q < 15) {
#pragma unroll
          for (int a = 0; a < 4; ++a) afn[a] = *reinterpret_cast<const float2*>(&xt[aoff[a] + 4 * (q + 1)]);
        } else if (tap < 8) {
#pragma unroll
          for (int a = 0; a < 4; ++a) afn[a] = *reinterpret_cast<const float2*>(&xn[aoff[a]]);
        }
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int a = 0; a < 4; ++a) {
            const float av = s ? afc[a].y : afc[a].x;
            acc[a][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, s ? b0.y : b0.x, acc[a][0], 0, 0, 0);
            acc[a][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, s ? b1.y : b1.x, acc[a][1], 0, 0, 0);
          }
#pragma unroll
        for (int a = 0; a < 4; ++a) afc[a] = afn[a];
      }
    }
    __syncthreads();                                  // buffer handed back to the gather waves
  }
  float* dst = partial + ((size_t)grp * 2 + slot) * PC_FRAG + (size_t)wv * (PC_FRAG / PC_WAVES);
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[((a * 2 + b) * 16 + r) * 64 + lane] = acc[a][b][r];
}

// ---------------------------------------------------------------------------------------------
// bf16 form (config 3's mixed precision: the reference autocasts the fusion features,
// volumetric_fusionnet.py:105-114): the same atoms, gather waves and stream-K ranges, with the
// halo samples rounded to bf16 in LDS and the MFMA on v_mfma_f32_32x32x16_bf16 (fp32
// accumulation; 16x the fp32 rate).  K = 16 per instruction: one (tap, 16-channel chunk) step is
// 8 MFMAs per compute wave (4 pixel blocks x 2 output blocks); lane (r, h) of a pixel block reads
// the 8 channels 16q + 8h .. +7 of its halo position (one 16-B LDS read).  Weights: the fragment
// copy `vfd_proj_conv_weight_bf16`: [D][9 taps][Cv/16][O/32 blocks][64 lanes][8], lane (r, h) of
// block ob holding W[o = 32 ob + r][c = 16 q + 8 h + j] (rounded to nearest even).
constexpr int PCB_XS = PC_CV + 8;               // bf16 per LDS row (144 B: 16-B aligned, staggered banks)
constexpr int PCB_ITERS = 9 * (PC_CV / 16);     // (tap, 16-channel chunk) steps per atom
#ifndef VFD_PCB_PF
#define VFD_PCB_PF 2
#endif
constexpr int PCB_PF = VFD_PCB_PF;              // weight-fragment prefetch distance (steps; 4 spills)

__global__ __launch_bounds__(PC_THREADS, 2) void pcvb_main_k(vfd_voxel_desc d, PcGeom g,
                                                            const float* __restrict__ vox,
                                                            const float* __restrict__ invK,
                                                            const float* __restrict__ E,
                                                            const bf16x8* __restrict__ Wq,
                                                            float* __restrict__ partial,
                                                            __bf16* __restrict__ xout) {
  __shared__ __attribute__((aligned(16))) __bf16 xs[2][PC_NPOS * PCB_XS];
  __shared__ PcTri tri[PC_WAVES][PC_GPOS];
  const int grp = blockIdx.x;
  const int a_lo = pc_lo(g, grp), a_hi = pc_lo(g, grp + 1);
  if (a_lo >= a_hi) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int V = d.X * d.Y * d.Z;
  const bool compute = wv < PC_WAVES;
  auto gather = [&](int atom, __bf16* dst) {
    const PcAtom a = pc_atom(d, g, atom);
    __bf16* xo = (xout && !VFD_PCVB_XO_COMPUTE) ? xout + (size_t)a.bc * (d.h + 2) * (d.w + 2) * d.D * PC_CV : nullptr;
    pc_gather<__bf16, PCB_XS>(d, dst, tri[wv - PC_WAVES], vox + (size_t)(a.bc / d.N) * V * PC_CV,
                              invK + a.bc * 16, E + a.bc * 16, a.y0, a.x0, a.di, wv - PC_WAVES, xo);
  };
  if (!compute) gather(a_lo, xs[0]);
  __syncthreads();
  if (!compute) {
    for (int atom = a_lo; atom < a_hi; ++atom) {
      if (atom + 1 < a_hi) gather(atom + 1, xs[(atom + 1 - a_lo) & 1]);
      __syncthreads();
    }
    return;
  }
  const int li = lane & 31, lh = lane >> 5;
  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  // LDS offset of the lane's A row at tap (0, 0), + 8h; pixel block a adds 32 pixels = exactly
  // two tile rows, a compile-time offset
  const int aoff0 = ((li >> 4) * PC_HC + (li & 15)) * PCB_XS + 8 * lh;
  constexpr int ABLK = 2 * PC_HC * PCB_XS;
  // weight fragments of the flattened (atom, step) stream, PCB_PF steps ahead
  // running pointer into the weight stream: one (tap, chunk) step = 8 blocks x 64 lanes; the next
  // depth bin follows contiguously, except after the last bin (back to bin 0)
  const bf16x8* wbase = Wq + (size_t)(2 * wv) * 64 + lane;
  const bf16x8* wp = wbase + (size_t)(a_lo % d.D) * PCB_ITERS * (PC_O / 32) * 64;
  const bf16x8* wend = wbase + (size_t)d.D * PCB_ITERS * (PC_O / 32) * 64;
  bf16x8 bq[PCB_PF][2];
  int pf_left = (a_hi - a_lo) * PCB_ITERS;         // steps still to prefetch
  auto prefetch = [&](int slot) {
    if (pf_left > 0) {
      bq[slot][0] = wp[0];
      bq[slot][1] = wp[64];
      wp += (PC_O / 32) * 64;
      if (wp == wend) wp = wbase;
      --pf_left;
    }
  };
#pragma unroll
  for (int k = 0; k < PCB_PF; ++k) prefetch(k);
  int slot = 0;
  int tile = a_lo / d.D;
  for (int atom = a_lo; atom < a_hi; ++atom) {
    const int t = atom / d.D;
    if (t != tile) {                                  // flush the finished tile's partial
      float* dst = partial + ((size_t)grp * 2 + slot) * PC_FRAG + (size_t)wv * (PC_FRAG / PC_WAVES);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            dst[((a * 2 + b) * 16 + r) * 64 + lane] = acc[a][b][r];
            acc[a][b][r] = 0.f;
          }
      slot = 1;
      tile = t;
    }
    const __bf16* xb = xs[(atom - a_lo) & 1];
    // A fragments software-pipelined one step ahead (LDS latency off the MFMA path)
    bf16x8 afc[4], afn[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) afc[a] = *reinterpret_cast<const bf16x8*>(&xb[aoff0 + a * ABLK]);
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap - 3 * ky;
      const __bf16* xt = xb + (ky * PC_HC + kx) * PCB_XS;
      const int tn = tap + 1, kyn = tn / 3, kxn = tn - 3 * kyn;
      const __bf16* xn = xb + (kyn * PC_HC + kxn) * PCB_XS;      // next tap (unused after tap 8)
#pragma unroll
      for (int q = 0; q < PC_CV / 16; ++q) {
        const int ring = q % PCB_PF;                  // (PC_CV / 16) % PCB_PF == 0: static ring slots
        const bf16x8 b0 = bq[ring][0], b1 = bq[ring][1];
        prefetch(ring);
        if (q < PC_CV / 16 - 1) {
#pragma unroll
          for (int a = 0; a < 4; ++a) afn[a] = *reinterpret_cast<const bf16x8*>(&xt[aoff0 + a * ABLK + 16 * (q + 1)]);
        } else if (tap < 8) {
#pragma unroll
          for (int a = 0; a < 4; ++a) afn[a] = *reinterpret_cast<const bf16x8*>(&xn[aoff0 + a * ABLK]);
        }
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          acc[a][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afc[a], b0, acc[a][0], 0, 0, 0);
          acc[a][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afc[a], b1, acc[a][1], 0, 0, 0);
        }
#pragma unroll
        for (int a = 0; a < 4; ++a) afc[a] = afn[a];
      }
    }
#if VFD_PCVB_XO_COMPUTE
    if (xout) {
      // the frustum side output (K3's layout, reflect copies included) for the weight gradient,
      // written by the compute waves from the staged image after this atom's MFMAs: the gather
      // waves bound the bf16 kernel (0.18 ms of its 0.99 at config 3 were these stores), the
      // compute waves wait for them at the barrier anyway.  Same bf16 values as the gather's.
      const PcAtom pa = pc_atom(d, g, atom);
      __bf16* xo = xout + (size_t)pa.bc * (d.h + 2) * (d.w + 2) * d.D * PC_CV;
      const int wo = d.w + 2;
      for (int e = threadIdx.x; e < PC_PIX * (PC_CV / 8); e += PC_WAVES * 64) {
        const int px = e >> 3, k = e & 7;                 // tile position, channel octet
        const int ty = px / PC_TC, tx = px - ty * PC_TC;
        const int py = pa.y0 + ty, pxx = pa.x0 + tx;
        if (py >= d.h || pxx >= d.w) continue;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(&xb[((ty + 1) * PC_HC + tx + 1) * PCB_XS + 8 * k]);
        int rows[3], cols[3], nr, nc;
        pad_sets(py, d.h, true, rows, &nr);
        pad_sets(pxx, d.w, true, cols, &nc);
        for (int r = 0; r < nr; ++r)
          for (int c = 0; c < nc; ++c)
            *reinterpret_cast<bf16x8*>(xo + (((size_t)rows[r] * wo + cols[c]) * d.D + pa.di) * PC_CV + 8 * k) = v;
      }
    }
#endif
    __syncthreads();                                  // buffer handed back to the gather waves
  }
  float* dst = partial + ((size_t)grp * 2 + slot) * PC_FRAG + (size_t)wv * (PC_FRAG / PC_WAVES);
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[((a * 2 + b) * 16 + r) * 64 + lane] = acc[a][b][r];
}

// Sum of each tile's partials (in workgroup order) + bias, LeakyReLU(0.1), stored into the
// reflect-padded NHWC map out [B*N, h+2, w+2, O] (the input of reduce_dim's second conv).
constexpr int PC_MAXC = 72;     // contributors of one tile (<= D + 1, D <= 64)
constexpr int PC_FSL = 8;       // fragment slices per tile (grid.y of the reduce kernels)
template <typename TO>
__global__ __launch_bounds__(256) void pcv_reduce_k(vfd_voxel_desc d, PcGeom g, const float* __restrict__ partial,
                                                    const float* __restrict__ bias, TO* __restrict__ out) {
  __shared__ int contrib[PC_MAXC];
  __shared__ int ncontrib;
  const int t = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int a0 = t * d.D, a1 = a0 + d.D;
  if (threadIdx.x == 0) {
    // workgroups whose atom range meets [a0, a1), in order; the first is the one containing a0
    int gg = (int)(((long long)a0 * g.ngroup) / g.natom);
    while (gg > 0 && pc_lo(g, gg) > a0) --gg;
    while (pc_lo(g, gg + 1) <= a0) ++gg;
    int n = 0;
    for (; gg < g.ngroup && n < PC_MAXC; ++gg) {
      const int lo = pc_lo(g, gg), hi = pc_lo(g, gg + 1);
      if (lo >= a1) break;
      if (hi <= a0 || lo >= hi) continue;
      contrib[n++] = gg * 2 + (lo >= a0 ? 0 : 1);   // slot 0 iff the tile is the group's first
    }
    ncontrib = n;
  }
  __syncthreads();
  const int nc = ncontrib;
  const int bc = t / g.tiles_img, ti = t - bc * g.tiles_img;
  const int y0 = (ti / g.tc) * PC_TR, x0 = (ti % g.tc) * PC_TC;
  const int ho = d.h + 2, wo = d.w + 2;
  TO* ob = out + (size_t)bc * ho * wo * PC_O;
  constexpr int FPS = 4 * 2 * 16 / PC_FSL;
  constexpr int U = 4;
  for (int fu = blockIdx.y * FPS; fu < (blockIdx.y + 1) * FPS; fu += U) {
    float su[U];
    frag_sums<U>(partial, contrib, nc, PC_FRAG, (size_t)wv * (PC_FRAG / PC_WAVES) + (fu * 64 + lane), su);
#pragma unroll
    for (int u = 0; u < U; ++u) {
    const int f = fu + u;
    const float s = su[u];
    const int a = f >> 5, bb = (f >> 4) & 1, r = f & 15;
    // fragment -> (pixel, channel): C/D layout of v_mfma_f32_32x32x2_f32
    const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    const int ip = 32 * a + row;
    const int o = wv * 64 + bb * 32 + (lane & 31);
    const int py = y0 + (ip >> 4), px = x0 + (ip & 15);
    if (py >= d.h || px >= d.w) continue;
    float v = s + bias[o];
    v = v > 0.f ? v : v * 0.1f;
    int rows[3], cols[3], nr, ncol;
    pad_sets(py, d.h, true, rows, &nr);
    pad_sets(px, d.w, true, cols, &ncol);
    for (int i = 0; i < nr; ++i)
      for (int j = 0; j < ncol; ++j) ob[((size_t)rows[i] * wo + cols[j]) * PC_O + o] = (TO)v;
    }
  }
}

static int pc_resident() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  return cus * PC_WG_PER_CU;
}

// Workgroup count: a multiple of the resident capacity, large enough that no range exceeds D
// atoms (so a range touches at most two tiles: partial slots 0 and 1).
static PcGeom pc_plan(const vfd_voxel_desc& d) {
  PcGeom g = pc_geom(d, 1);
  const int res = pc_resident();
  const int need = (g.natom + d.D - 1) / d.D;
  g.ngroup = res * ((need + res - 1) / res);
  return g;
}

// =============================================================================================
// K3C data gradient — reduce_dim's first conv, backward w.r.t. its reflect-padded input (the
// frustum features K3's backward consumes), as an fp32 MFMA GEMM over the padded grid:
//
//   dXp[bc, Y, X, n] = sum_{ty, tx, o} G[bc, Y - ty, X - tx, o] * W[o, n, ty, tx]
//
// G = d pre-activation [B*N, h, w, O] (zero outside the h x w grid), n = d*Cv + c (K3's channel
// order).  M = padded positions of ALL cameras, flattened (row-major, 128 per tile): the cameras'
// (h+2)-row padded grids are stacked into one tall grid of B*N*(h+2) rows, on which camera bc's
// G rows y < h sit at virtual rows bc*(h+2) + y and rows h, h+1 are zero, so a tap reaching above
// a camera's first row reads the previous camera's two zero rows — the stacked problem is exactly
// the B*N per-camera ones, with one ragged tile in total instead of one per camera (config 2:
// 193 tiles of 128 for 24 600 positions, 3 % fewer than 6 x 33).  N = D*Cv (256 per tile,
// zero-padded weights past D*Cv), K = 9 taps x O.  An atom = (tile, 32-channel chunk of O): the loader waves
// stage the chunk's G rows under the tile (<= hrows rows x (w + 4) columns, zero margins) in LDS
// while the compute waves run the previous atom's 9 taps x 8 channel quads (same wave roles and
// fragment pipeline as the forward).  Stream-K over atoms: a tile whole inside one workgroup's
// range is stored directly; the (at most two) split tiles of a range go to partial slots that
// `pcd_reduce_k` sums in workgroup order (deterministic).
#ifndef VFD_PD_PF
#define VFD_PD_PF 4
#endif
constexpr int PD_PF = VFD_PD_PF;                // weight-fragment prefetch distance of the data gradient
constexpr int PD_OC = 32;                       // O channels per atom
constexpr int PD_XS = PD_OC + 4;                // LDS floats per staged position
constexpr int PD_N = PC_WAVES * 64;             // n per tile
constexpr int PD_CHUNKS = PC_O / PD_OC;         // atoms per tile
constexpr int PD_ITERS = 9 * (PD_OC / 4);       // (tap, quad) iterations per atom
constexpr int PD_LDS_MAX = 160 * 1024;

struct PdGeom {
  int nbc, h, w, wo, npix, mtot, mtiles, ntot, np, ntile, natom, ngroup, hrows, cols, lds_floats;
};

__host__ __device__ inline int pd_lo(const PdGeom& g, int grp) {
  return (int)(((long long)grp * g.natom) / g.ngroup);
}

struct PdTile {
  int nt, mt, m0, ymin;
};

// tile order: n-tile outermost (a workgroup's consecutive tiles share the n-tile's weights);
// m0 / ymin are positions / rows of the stacked grid
__device__ __forceinline__ PdTile pd_tile(const PdGeom& g, int t) {
  PdTile r;
  r.mt = t % g.mtiles;
  r.nt = t / g.mtiles;
  r.m0 = r.mt * PC_PIX;
  r.ymin = r.m0 / g.wo;
  return r;
}

// loader waves (tid 0..255): stacked G rows ymin-2 .. ymin-2+hrows-1, columns -2 .. w+1, channels
// of chunk ch (zero outside a camera's h x w grid)
__device__ __forceinline__ void pd_stage(const PdGeom& g, float* __restrict__ dst, const float* __restrict__ gp,
                                         int atom, int tid) {
  const int t = atom / PD_CHUNKS, ch = atom - t * PD_CHUNKS;
  const PdTile tl = pd_tile(g, t);
  const int npos = g.hrows * g.cols;
  const int q = tid & 7;
  const int hp = g.h + 2;
  const float* src = gp + ch * PD_OC + 4 * q;
  for (int p0 = tid >> 3; p0 < npos; p0 += 4 * 32) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = p0 + 32 * u;
      const int hr = p / g.cols, c = p - hr * g.cols;
      const int r = tl.ymin - 2 + hr, x = c - 2;
      const int bc = r >= 0 ? r / hp : 0, y = r - bc * hp;
      v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p < npos && r >= 0 && bc < g.nbc && y < g.h && x >= 0 && x < g.w)
        v[u] = *reinterpret_cast<const float4*>(src + (((size_t)bc * g.h + y) * g.w + x) * PC_O);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = p0 + 32 * u;
      if (p < npos) *reinterpret_cast<float4*>(dst + p * PD_XS + 4 * q) = v[u];
    }
  }
}

// Weight layout Wd: [9 taps (flipped: tap' = (2-ty)*3 + (2-tx))][O/4 quads][np][2 (h)][2 (s)],
// o = 4*quad + 2*h + s, n = d*Cv + c (zero for n >= D*Cv).
__global__ __launch_bounds__(PC_THREADS, 2) void pcd_main_k(PdGeom g, const float* __restrict__ gp,
                                                           const float* __restrict__ Wd,
                                                           float* __restrict__ dx,
                                                           float* __restrict__ partial) {
  extern __shared__ float pd_lds[];
  // XCD-contiguous ranges: workgroups are dealt round-robin to the 8 XCDs, so logical group
  // (blockIdx % 8) * (G / 8) + blockIdx / 8 gives each XCD one contiguous run of tiles — a
  // 1-2 n-tile window of weights (2.4 MB each) that stays in that XCD's L2 while its M-tiles pass
  const int grp = (g.ngroup % 8 == 0) ? (blockIdx.x % 8) * (g.ngroup / 8) + blockIdx.x / 8 : blockIdx.x;
  const int a_lo = pd_lo(g, grp), a_hi = pd_lo(g, grp + 1);
  if (a_lo >= a_hi) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool compute = wv < PC_WAVES;
  if (!compute) pd_stage(g, pd_lds, gp, a_lo, threadIdx.x - 64 * PC_WAVES);
  __syncthreads();
  if (!compute) {
    for (int atom = a_lo; atom < a_hi; ++atom) {
      if (atom + 1 < a_hi)
        pd_stage(g, pd_lds + ((atom + 1 - a_lo) & 1) * g.lds_floats, gp, atom + 1, threadIdx.x - 64 * PC_WAVES);
      __syncthreads();
    }
    return;
  }
  const int li = lane & 31, lh = lane >> 5;
  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const float2* wlane = reinterpret_cast<const float2*>(Wd) + (size_t)(wv * 64 + li) * 2 + lh;
  float2 bq[PD_PF][2];
  int pf_atom = a_lo, pf_it = 0;
  auto prefetch = [&](int slot) {
    if (pf_atom < a_hi) {
      const int t = pf_atom / PD_CHUNKS, ch = pf_atom - t * PD_CHUNKS;
      const int nt = t / g.mtiles;
      const int tap = pf_it >> 3, q = pf_it & 7;
      const float2* w = wlane + ((size_t)(tap * (PC_O / 4) + ch * (PD_OC / 4) + q) * g.np + nt * PD_N) * 2;
      bq[slot][0] = w[0];
      bq[slot][1] = w[64];
      if (++pf_it == PD_ITERS) { pf_it = 0; ++pf_atom; }
    }
  };
#pragma unroll
  for (int k = 0; k < PD_PF; ++k) prefetch(k);
  for (int atom = a_lo; atom < a_hi; ++atom) {
    const int t = atom / PD_CHUNKS, ch = atom - t * PD_CHUNKS;
    const PdTile tl = pd_tile(g, t);
    int aoff[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      int m = tl.m0 + 32 * a + li;
      m = m < g.mtot ? m : g.mtot - 1;                 // rows past the grid: computed, never stored
      const int Y = m / g.wo, X = m - Y * g.wo;
      aoff[a] = ((Y - tl.ymin) * g.cols + X) * PD_XS + 2 * lh;
    }
    const float* xb = pd_lds + ((atom - a_lo) & 1) * g.lds_floats;
    float2 afc[4], afn[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) afc[a] = *reinterpret_cast<const float2*>(&xb[aoff[a]]);
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap - 3 * ky;
      const float* xt = xb + (ky * g.cols + kx) * PD_XS;
      const int tn = tap + 1, kyn = tn / 3, kxn = tn - 3 * kyn;
      const float* xn = xb + (kyn * g.cols + kxn) * PD_XS;
#pragma unroll
      for (int q = 0; q < PD_OC / 4; ++q) {
        const int ring = q % PD_PF;
        const float2 b0 = bq[ring][0], b1 = bq[ring][1];
        prefetch(ring);
        if (q < PD_OC / 4 - 1) {
#pragma unroll
          for (int a = 0; a < 4; ++a) afn[a] = *reinterpret_cast<const float2*>(&xt[aoff[a] + 4 * (q + 1)]);
        } else if (tap < 8) {
#pragma unroll
          for (int a = 0; a < 4; ++a) afn[a] = *reinterpret_cast<const float2*>(&xn[aoff[a]]);
        }
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int a = 0; a < 4; ++a) {
            const float av = s ? afc[a].y : afc[a].x;
            acc[a][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, s ? b0.y : b0.x, acc[a][0], 0, 0, 0);
            acc[a][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, s ? b1.y : b1.x, acc[a][1], 0, 0, 0);
          }
#pragma unroll
        for (int a = 0; a < 4; ++a) afc[a] = afn[a];
      }
    }
    __syncthreads();                                  // buffer handed back to the loader waves
    if (ch == PD_CHUNKS - 1 || atom == a_hi - 1) {
      const int ts = t * PD_CHUNKS;
      if (ts >= a_lo && ts + PD_CHUNKS <= a_hi) {     // whole tile in this range: store
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int n = tl.nt * PD_N + wv * 64 + b * 32 + li;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int m = tl.m0 + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * lh;
              if (m < g.mtot && n < g.ntot) dx[(size_t)m * g.ntot + n] = acc[a][b][r];
              acc[a][b][r] = 0.f;
            }
          }
      } else {                                        // split tile: partial slot
        const int slot = t == a_lo / PD_CHUNKS ? 0 : 1;
        float* dst = partial + ((size_t)grp * 2 + slot) * PC_FRAG + (size_t)wv * (PC_FRAG / PC_WAVES);
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              dst[((a * 2 + b) * 16 + r) * 64 + lane] = acc[a][b][r];
              acc[a][b][r] = 0.f;
            }
      }
    }
  }
}

// Ranges hold >= PD_CHUNKS atoms, so a split tile contains exactly one group boundary lo(g):
// workgroup (g, slice) sums group g-1's and group g's partials of that tile, in that order.
__global__ __launch_bounds__(256) void pcd_reduce_k(PdGeom g, const float* __restrict__ partial,
                                                    float* __restrict__ dx) {
  const int grp = blockIdx.x;
  const int lo = pd_lo(g, grp);
  if (grp == 0 || lo % PD_CHUNKS == 0) return;        // boundary on a tile edge: nothing split
  const int t = lo / PD_CHUNKS;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c0 = (grp - 1) * 2 + (t == pd_lo(g, grp - 1) / PD_CHUNKS ? 0 : 1), c1 = grp * 2;
  const PdTile tl = pd_tile(g, t);
  constexpr int FPS = 4 * 2 * 16 / PC_FSL;
  constexpr int U = 4;
  const int contrib[2] = {c0, c1};
  for (int fu = blockIdx.y * FPS; fu < (blockIdx.y + 1) * FPS; fu += U) {
    float su[U];
    frag_sums<U>(partial, contrib, 2, PC_FRAG, (size_t)wv * (PC_FRAG / PC_WAVES) + (fu * 64 + lane), su);
#pragma unroll
    for (int u = 0; u < U; ++u) {
    const int f = fu + u;
    const int a = f >> 5, bb = (f >> 4) & 1, r = f & 15;
    const float s = su[u];
    const int m = tl.m0 + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    const int n = tl.nt * PD_N + wv * 64 + bb * 32 + (lane & 31);
    if (m < g.mtot && n < g.ntot) dx[(size_t)m * g.ntot + n] = s;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Folded form (vfd_voxel_desc.pad_out == 2): the data gradient of the reflect-padded input with the
// reflect-pad adjoint folded in, so only the h x w interior is computed.  A padded border position's
// gradient belongs to its mirror pixel (pad_sets); with the flipped taps,
//   dX[y=1]    = dXp[2] + dXp[0],        dXp[0]   = G[0] W_(ky=2)     (only that tap row reaches G)
//   dX[y=h-2]  = dXp[h-1] + dXp[h+1],    dXp[h+1] = G[h-1] W_(ky=0)
// (columns alike), i.e. the A operand of row 1 at ky = 2 is G[2] + G[0] and of row h-2 at ky = 0 is
// G[h-3] + G[h-1].  Column folds ride in two extra staged columns per row (E1 = G[.][2] + G[.][0]
// read by x = 1 at kx = 2, E2 = G[.][w-3] + G[.][w-1] by x = w-2 at kx = 0); the row fold in one
// extra staged row per tile (a tile spans <= 3 pixel rows, so with h >= 6 it holds row 1 or row h-2,
// never both), read by those lanes at those taps instead of their plain row — one A read per lane
// as in the padded form; the fold row's E columns carry the corner terms.  Tiles are 128 consecutive interior pixels of ONE camera (config 2:
// 30 per camera, 180 in all against 193 padded ones), written into the interior of the padded
// layout; K3's backward then reads every sample straight from it (its plan built with pad_out = 2:
// no fold buffer, no fold launch).
// When at most half of the last n-tile is real frustum channels (config 2: 3 200 = 12.5 x 256),
// that n-tile's atoms [nfa, natom) run in the half-width form (each wave 32 channels, one MFMA
// n-block, instead of 64), so the zero padding costs no MFMAs.  Groups [0, gfull) split the
// full-width atoms [0, nfa), groups [gfull, ngroup) the half-width ones, the two counts in
// proportion to the two regions' MFMA work, so every group (one per CU) finishes together.
// No half-width region: nfa = natom, gfull = ngroup.
struct PfGeom {
  int nbc, h, w, ntot, np, tpc, mtiles, ntile, natom, ngroup, hrows, cols, lds_floats, nfa, gfull;
};
#ifndef VFD_PF_HBIAS
#define VFD_PF_HBIAS 2          // half-width groups beyond their rounded-up share: 0 / 1 / 2 / 4 -> 2.803 / 2.787 / 2.760 / 2.767 ms (one box, C-ABI micro)
#endif

__host__ __device__ inline int pf_lo(const PfGeom& g, int grp) {
  if (grp <= g.gfull) return (int)(((long long)grp * g.nfa) / g.gfull);
  return g.nfa + (int)(((long long)(grp - g.gfull) * (g.natom - g.nfa)) / (g.ngroup - g.gfull));
}

struct PfTile {
  int nt, bc, m0, y0;
};

__device__ __forceinline__ PfTile pf_tile(const PfGeom& g, int t) {
  PfTile r;
  const int mt = t % g.mtiles;
  r.nt = t / g.mtiles;
  r.bc = mt / g.tpc;
  r.m0 = (mt - r.bc * g.tpc) * PC_PIX;
  r.y0 = r.m0 / g.w;
  return r;
}

// one staged element: G row y (zero outside [0, h)) at staged column c (G column c - 2; E1 / E2)
__device__ __forceinline__ float4 pf_elem(const PfGeom& g, const float* __restrict__ src, int y, int c) {
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (y < 0 || y >= g.h) return v;
  const float* row = src + (size_t)y * g.w * PC_O;
  if (c < g.w + 4) {
    const int x = c - 2;
    if (x >= 0 && x < g.w) v = *reinterpret_cast<const float4*>(row + (size_t)x * PC_O);
  } else {
    const int xa = c == g.w + 4 ? 2 : g.w - 3, xb = c == g.w + 4 ? 0 : g.w - 1;
    const float4 a = *reinterpret_cast<const float4*>(row + (size_t)xa * PC_O);
    const float4 b = *reinterpret_cast<const float4*>(row + (size_t)xb * PC_O);
    v = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  }
  return v;
}

// loader waves (tid 0..255): staged row r < hrows = G row y0 - 1 + r of the tile's camera,
// columns 0 .. w+3 = G columns -2 .. w+1, then E1, E2; row hrows = the tile's fold row (G[2] + G[0]
// when the tile holds pixel row 1, G[h-3] + G[h-1] when it holds row h-2; h >= 6: never both);
// channels of chunk ch
__device__ __forceinline__ void pf_stage(const PfGeom& g, float* __restrict__ dst, const float* __restrict__ gp,
                                         int atom, int tid) {
  const int t = atom / PD_CHUNKS, ch = atom - t * PD_CHUNKS;
  const PfTile tl = pf_tile(g, t);
  const int hw = g.h * g.w;
  const int ylast = (tl.m0 + PC_PIX - 1 < hw ? tl.m0 + PC_PIX - 1 : hw - 1) / g.w;
  const int fa = tl.y0 <= 1 && ylast >= 1 ? 2 : (tl.y0 <= g.h - 2 && ylast >= g.h - 2 ? g.h - 3 : -1);
  const int fb = fa == 2 ? 0 : g.h - 1;
  const int npos = (g.hrows + (fa >= 0 ? 1 : 0)) * g.cols;
  const int q = tid & 7;
  const float* src = gp + (size_t)tl.bc * g.h * g.w * PC_O + ch * PD_OC + 4 * q;
  for (int p0 = tid >> 3; p0 < npos; p0 += 4 * 32) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = p0 + 32 * u;
      const int hr = p / g.cols, c = p - hr * g.cols;
      v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p < npos) {
        if (hr < g.hrows) {
          v[u] = pf_elem(g, src, tl.y0 - 1 + hr, c);
        } else {
          const float4 a = pf_elem(g, src, fa, c), b = pf_elem(g, src, fb, c);
          v[u] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = p0 + 32 * u;
      if (p < npos) *reinterpret_cast<float4*>(dst + p * PD_XS + 4 * q) = v[u];
    }
  }
}

template <bool HALF>
__device__ __forceinline__ void pcdf_body(const PfGeom& g, int grp, const float* __restrict__ gp,
                                          const float* __restrict__ Wd, float* __restrict__ dx,
                                          float* __restrict__ partial, float* __restrict__ pd_lds) {
  const int a_lo = pf_lo(g, grp), a_hi = pf_lo(g, grp + 1);
  if (a_lo >= a_hi) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool compute = wv < PC_WAVES;
  if (!compute) pf_stage(g, pd_lds, gp, a_lo, threadIdx.x - 64 * PC_WAVES);
  __syncthreads();
  if (!compute) {
    for (int atom = a_lo; atom < a_hi; ++atom) {
      if (atom + 1 < a_hi)
        pf_stage(g, pd_lds + ((atom + 1 - a_lo) & 1) * g.lds_floats, gp, atom + 1, threadIdx.x - 64 * PC_WAVES);
      __syncthreads();
    }
    return;
  }
  const int li = lane & 31, lh = lane >> 5;
  const int hw = g.h * g.w;
  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  // Weight fragments by buffer loads: the lane's part is a constant voffset, the (atom, tap, quad)
  // part a uniform soffset.  The B fragments of step (tap, q) are loaded four steps ahead into ring
  // slot q & 3 (static slots: the unrolled quad loop needs no register rotation across the tap
  // loop's back edge), issued right after step q's MFMAs have read the slot; the next tap's / next
  // atom's items come from a base selected without a branch (the range's last atom re-reads its
  // own, in range and unused).  Round 6: no scalar branches in the tap loop (the per-step prefetch
  // bookkeeping split every quad step into several basic blocks, which kept the scheduler from
  // issuing the next A fragments' LDS reads before the MFMAs).
  constexpr int PFD_RING = 4;
  const unsigned npb = (unsigned)g.np * 16u;          // bytes between consecutive (tap, quad) items
  const __amdgpu_buffer_rsrc_t rs_w = __builtin_amdgcn_make_buffer_rsrc(
      (void*)Wd, 0, (int)(9u * (PC_O / 4) * npb), 0x00020000);
  const int voff = ((wv * 64 + li) * 2 + lh) * 8;
  auto wbase = [&](int at) {                          // byte offset of atom `at`'s (tap 0, quad 0) item
    const int t = at / PD_CHUNKS, ch = at - t * PD_CHUNKS;
    // wave-uniform (the division runs on the vector unit): readfirstlane keeps the buffer loads'
    // soffset scalar (a VGPR soffset compiles to a waterfall loop per load)
    // (half width: wave wv's channels wv * 32 + li instead of wv * 64 + li — the same lane offset
    // moved by a wave-uniform -512 * wv bytes, folded into the scalar base)
    return (unsigned)__builtin_amdgcn_readfirstlane(
        (int)((unsigned)(ch * (PD_OC / 4)) * npb + (unsigned)(t / g.mtiles) * (PD_N * 16u)) - (HALF ? 512 * wv : 0));
  };
  auto wload = [&](unsigned soff, float2 (&b)[2]) {
    const auto v0 = __builtin_amdgcn_raw_buffer_load_b64(rs_w, voff, (int)soff, 0);
    b[0] = make_float2(__uint_as_float(v0[0]), __uint_as_float(v0[1]));
    if (!HALF) {
      const auto v1 = __builtin_amdgcn_raw_buffer_load_b64(rs_w, voff + 512, (int)soff, 0);
      b[1] = make_float2(__uint_as_float(v1[0]), __uint_as_float(v1[1]));
    } else {
      b[1] = make_float2(0.f, 0.f);
    }
  };
  float2 bq[PFD_RING][2];
  unsigned cbase = wbase(a_lo);
#pragma unroll
  for (int q = 0; q < PFD_RING; ++q) wload(cbase + (unsigned)q * npb, bq[q]);
  constexpr int NQ = PD_OC / 4;                       // quads per tap (8)
  int cur_t = -1;
  int pyx[4];                                         // (row << 16) | column of the lane's pixels
  for (int atom = a_lo; atom < a_hi; ++atom) {
    const int t = atom / PD_CHUNKS, ch = atom - t * PD_CHUNKS;
    const PfTile tl = pf_tile(g, t);
    const unsigned nbase = atom + 1 < a_hi ? wbase(atom + 1) : cbase;
    if (t != cur_t) {                                 // pixel geometry once per tile (8 atoms)
      cur_t = t;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        int m = tl.m0 + 32 * a + li;
        m = m < hw ? m : hw - 1;                      // pixels past the camera: computed, never stored
        const int y = m / g.w;
        pyx[a] = (y << 16) | (m - y * g.w);
      }
    }
    const float* xb = pd_lds + ((atom - a_lo) & 1) * g.lds_floats;
    // per-lane LDS offset of tap `tap`: the A row (the fold row for row 1 at ky = 2 and row h-2 at
    // ky = 0) and column (E1 / E2 for the column folds).  Plain position: base + the tap's uniform
    // (ky, kx) step; a fold replaces the column (px = 1 at kx = 2 -> E1 = column w+4, px = w-2 at
    // kx = 0 -> E2 = column w+5) or the row (the staged fold row hrows) — uniform deltas per tap
    // and tile, added where the lane's pixel matches the tap's fold column / row
    auto offsets = [&](int tap, int* o1) {
      const int ky = tap / 3, kx = tap - 3 * ky;
      const int step = (ky * g.cols + kx) * PD_XS;
      const int fcol = kx == 2 ? 1 : (kx == 0 ? g.w - 2 : -1);
      const int dcol = (kx == 2 ? g.w : 6) * PD_XS;
      const int frow = ky == 2 ? 1 : (ky == 0 ? g.h - 2 : -1);
      const int drow = (g.hrows - (ky == 2 ? 3 - tl.y0 : g.h - 2 - tl.y0)) * g.cols * PD_XS;
      const int r1 = g.cols * PD_XS, r2 = 2 * g.cols * PD_XS;   // a tile's pixels sit in rows y0 .. y0+2
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int px = pyx[a] & 0xFFFF, py = pyx[a] >> 16, dy = py - tl.y0;
        const int rowo = dy == 0 ? 0 : (dy == 1 ? r1 : r2);
        o1[a] = rowo + (px + 1) * PD_XS + 2 * lh + step + (px == fcol ? dcol : 0) + (py == frow ? drow : 0);
      }
    };
    int o1c[4];
    offsets(0, o1c);
    float2 afc[4], afn[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) afc[a] = *reinterpret_cast<const float2*>(&xb[o1c[a]]);
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      // refill items: (tap, q + 4) for q < 4; (tap + 1, q - 4) of this atom, or of the next at tap 8
      const unsigned tb = (unsigned)__builtin_amdgcn_readfirstlane((int)(cbase + (unsigned)(tap * (PC_O / 4)) * npb));
      const unsigned nb = (unsigned)__builtin_amdgcn_readfirstlane((int)(tap < 8 ? tb + (unsigned)(PC_O / 4) * npb : nbase));
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        if (q < NQ - 1) {
#pragma unroll
          for (int a = 0; a < 4; ++a) afn[a] = *reinterpret_cast<const float2*>(&xb[o1c[a] + 4 * (q + 1)]);
        } else {                                      // the next tap's first quad (tap 8: unused)
          offsets(tap < 8 ? tap + 1 : 8, o1c);
#pragma unroll
          for (int a = 0; a < 4; ++a) afn[a] = *reinterpret_cast<const float2*>(&xb[o1c[a]]);
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int a = 0; a < 4; ++a) {
            const float v = s2 ? afc[a].y : afc[a].x;
            acc[a][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(v, s2 ? bq[q & 3][0].y : bq[q & 3][0].x, acc[a][0], 0, 0, 0);
            if (!HALF)
              acc[a][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(v, s2 ? bq[q & 3][1].y : bq[q & 3][1].x, acc[a][1], 0, 0, 0);
          }
        wload(q < 4 ? tb + (unsigned)(q + 4) * npb : nb + (unsigned)(q - 4) * npb, bq[q & 3]);
        // in this step: the next A fragments' LDS reads first, then the 16 (half: 8) MFMAs, then the refill
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);             // DS read
        __builtin_amdgcn_sched_group_barrier(0x008, HALF ? 8 : 16, 0); // MFMA
        __builtin_amdgcn_sched_group_barrier(0x020, HALF ? 1 : 2, 0);  // VMEM read
#pragma unroll
        for (int a = 0; a < 4; ++a) afc[a] = afn[a];
      }
    }
    cbase = nbase;
    __syncthreads();                                  // buffer handed back to the loader waves
    if (ch == PD_CHUNKS - 1 || atom == a_hi - 1) {
      const int ts = t * PD_CHUNKS;
      if (ts >= a_lo && ts + PD_CHUNKS <= a_hi) {     // whole tile in this range: store
        // the tile's 128 pixels span <= 3 rows from y0 (w >= 64): row / column by two compares;
        // element indices within the camera in 32 bits (pf_supported: one camera's padded map < 2^32)
        const int mr0 = tl.m0 - tl.y0 * g.w;          // the tile's first pixel within row y0
        float* dcam = dx + (size_t)tl.bc * (g.h + 2) * (g.w + 2) * g.ntot;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int n = HALF ? (b ? g.ntot : tl.nt * PD_N + wv * 32 + li)       // half width: b = 1 none
                               : tl.nt * PD_N + wv * 64 + b * 32 + li;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int mo = 32 * a + (r & 3) + 8 * (r >> 2) + 4 * lh;
              const int mr = mr0 + mo;
              const int dy = (mr >= g.w ? 1 : 0) + (mr >= 2 * g.w ? 1 : 0);
              const int x = mr - dy * g.w;
              if (tl.m0 + mo < hw && n < g.ntot) {
                const unsigned e = ((unsigned)(tl.y0 + dy + 1) * (unsigned)(g.w + 2) + (unsigned)(x + 1)) *
                                   (unsigned)g.ntot + (unsigned)n;
                dcam[e] = acc[a][b][r];
              }
              acc[a][b][r] = 0.f;
            }
          }
      } else {                                        // split tile: partial slot
        const int slot = t == a_lo / PD_CHUNKS ? 0 : 1;
        float* dst = partial + ((size_t)grp * 2 + slot) * PC_FRAG + (size_t)wv * (PC_FRAG / PC_WAVES);
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              dst[((a * 2 + b) * 16 + r) * 64 + lane] = acc[a][b][r];
              acc[a][b][r] = 0.f;
            }
      }
    }
  }
}

__global__ __launch_bounds__(PC_THREADS, 2) void pcdf_main_k(PfGeom g, const float* __restrict__ gp,
                                                            const float* __restrict__ Wd,
                                                            float* __restrict__ dx,
                                                            float* __restrict__ partial) {
  extern __shared__ float pd_lds[];
  const int grp = (g.ngroup % 8 == 0) ? (blockIdx.x % 8) * (g.ngroup / 8) + blockIdx.x / 8 : blockIdx.x;
  if (grp < g.gfull)                                  // workgroup-uniform: one width per group
    pcdf_body<false>(g, grp, gp, Wd, dx, partial, pd_lds);
  else
    pcdf_body<true>(g, grp, gp, Wd, dx, partial, pd_lds);
}

__global__ __launch_bounds__(256) void pcdf_reduce_k(PfGeom g, const float* __restrict__ partial,
                                                     float* __restrict__ dx) {
  const int grp = blockIdx.x;
  const int lo = pf_lo(g, grp);
  if (grp == 0 || lo % PD_CHUNKS == 0) return;        // boundary on a tile edge: nothing split
  const int t = lo / PD_CHUNKS;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c0 = (grp - 1) * 2 + (t == pf_lo(g, grp - 1) / PD_CHUNKS ? 0 : 1), c1 = grp * 2;
  const PfTile tl = pf_tile(g, t);
  const int hw = g.h * g.w;
  constexpr int FPS = 4 * 2 * 16 / PC_FSL;
  constexpr int U = 4;
  const int contrib[2] = {c0, c1};
  for (int fu = blockIdx.y * FPS; fu < (blockIdx.y + 1) * FPS; fu += U) {
    float su[U];
    frag_sums<U>(partial, contrib, 2, PC_FRAG, (size_t)wv * (PC_FRAG / PC_WAVES) + (fu * 64 + lane), su);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int f = fu + u;
      const int a = f >> 5, bb = (f >> 4) & 1, r = f & 15;
      const int m = tl.m0 + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const int n = t >= g.nfa / PD_CHUNKS ? (bb ? g.ntot : tl.nt * PD_N + wv * 32 + (lane & 31))
                                           : tl.nt * PD_N + wv * 64 + bb * 32 + (lane & 31);
      if (m < hw && n < g.ntot) {
        const int y = m / g.w, x = m - y * g.w;
        dx[(((size_t)tl.bc * (g.h + 2) + y + 1) * (g.w + 2) + x + 1) * g.ntot + n] = su[u];
      }
    }
  }
}

static PfGeom pf_plan(const vfd_voxel_desc& d) {
  PfGeom g;
  g.nbc = d.B * d.N;
  g.h = d.h;
  g.w = d.w;
  g.ntot = d.D * PC_CV;
  g.np = (g.ntot + PD_N - 1) / PD_N * PD_N;
  g.tpc = (d.h * d.w + PC_PIX - 1) / PC_PIX;
  g.mtiles = g.nbc * g.tpc;
  g.ntile = (g.np / PD_N) * g.mtiles;
  g.natom = g.ntile * PD_CHUNKS;
  g.hrows = (d.w + PC_PIX - 2) / d.w + 3;             // G rows under 128 consecutive pixels + 2
  g.cols = d.w + 6;                                   // 2 + w + 2 columns, E1, E2
  g.lds_floats = (g.hrows + 1) * g.cols * PD_XS;      // + the fold row
  const int res = pc_resident();
  const int most = g.natom / PD_CHUNKS;
  g.ngroup = most < res ? (most > 0 ? most : 1) : res;
  g.nfa = g.natom;
  g.gfull = g.ngroup;
  const int nn = g.np / PD_N;
  if (g.ntot - (nn - 1) * PD_N <= PD_N / 2 && nn > 1 && g.ngroup > 1) {
    // the half-width n-tile: (nn - 1) full n-tiles against half a tile's work; each region's groups
    // keep >= PD_CHUNKS atoms (a tile then meets at most two groups)
    const int nfa = (nn - 1) * g.mtiles * PD_CHUNKS, nha = g.natom - nfa;
    // a half-width atom costs at least half a full one (same staging and LDS reads, half the
    // MFMAs): the share rounded up, plus VFD_PF_HBIAS groups, so the half-width groups are not the tail
    int gh = (int)(((long long)g.ngroup * nha + 2LL * nfa + nha - 1) / (2LL * nfa + nha)) + VFD_PF_HBIAS;
    gh = gh > nha / PD_CHUNKS ? nha / PD_CHUNKS : gh;
    const int gf = g.ngroup - gh;
    if (gh >= 1 && gf >= 1 && gf <= nfa / PD_CHUNKS) {
      g.nfa = nfa;
      g.gfull = gf;
    }
  }
  return g;
}


static bool pf_supported(const vfd_voxel_desc& d) {
  if (d.Cv != PC_CV || d.B <= 0 || d.N <= 0 || d.h < 6 || d.w < 3 || d.D <= 0 || d.D > 64) return false;
  const PfGeom g = pf_plan(d);
  if (g.hrows > 5) return false;                      // a tile spans <= 3 pixel rows (w >= 64)
  if ((size_t)(d.h + 2) * (d.w + 2) * g.ntot >= ((size_t)1 << 32)) return false;
  return (size_t)2 * g.lds_floats * sizeof(float) <= PD_LDS_MAX;
}

// one workgroup per CU, ranges of >= PD_CHUNKS atoms (a tile meets at most two groups per side)
static PdGeom pd_plan(const vfd_voxel_desc& d) {
  PdGeom g;
  g.nbc = d.B * d.N;
  g.h = d.h;
  g.w = d.w;
  g.wo = d.w + 2;
  g.npix = (d.h + 2) * g.wo;
  g.mtot = g.nbc * g.npix;
  g.mtiles = (g.mtot + PC_PIX - 1) / PC_PIX;
  g.ntot = d.D * PC_CV;
  g.np = (g.ntot + PD_N - 1) / PD_N * PD_N;
  g.ntile = (g.np / PD_N) * g.mtiles;
  g.natom = g.ntile * PD_CHUNKS;
  g.hrows = 3 + (g.wo + PC_PIX - 2) / g.wo;           // rows under 128 consecutive positions + 2
  g.cols = d.w + 4;
  g.lds_floats = g.hrows * g.cols * PD_XS;
  const int res = pc_resident();
  const int most = g.natom / PD_CHUNKS;
  g.ngroup = most < res ? (most > 0 ? most : 1) : res;
  return g;
}

static bool pd_supported(const vfd_voxel_desc& d) {
  if (d.Cv != PC_CV || d.B <= 0 || d.N <= 0 || d.h < 2 || d.w < 2 || d.D <= 0 || d.D > 64) return false;
  const PdGeom g = pd_plan(d);
  return (size_t)2 * g.lds_floats * sizeof(float) <= PD_LDS_MAX;
}

// =============================================================================================
// K3C data gradient, round 4 ("pcg"): the folded form (reflect-pad adjoint inside the GEMM, interior
// only, as pcdf) on tiles of 256 interior pixels x 128 frustum channels, fp32 and bf16.
//
// Each of the 4 compute waves owns 8 pixel blocks (256 pixels) x ONE 32-channel block of n, so a
// weight fragment feeds 8 pixel blocks (pcdf: 4) — half the weight bytes streamed from L2 per MFMA
// — and N = D*Cv = 3200 splits into 25 tiles of 128 with no zero padding (pcdf: 13 x 256, 4 %
// zero work).  Tiles are 256 consecutive interior pixels of one camera (config 2: 15 per camera,
// exact), whose staged G rows (the whole rows under the tile, columns -1 .. w, then the E1 / E2
// column folds) and both fold rows (F1 = G[2] + G[0] for pixel row 1 at ky' = 2, F2 = G[h-3] +
// G[h-1] for row h-2 at ky' = 0; staged only when the tile holds that row) fit LDS double-buffered
// for w <= 128 (config 5: w = 120, 158.7 KB), because an atom carries only OC output channels:
// fp32 16 (9 taps x 4 channel quads of v_mfma_f32_32x32x2_f32, 16 MFMAs per step), bf16 32 (9 taps
// x 2 sixteen-channel steps of v_mfma_f32_32x32x16_bf16, 8 MFMAs per step).  Same loader / compute
// wave split, stream-K ranges (>= OC atoms: a split tile meets two groups) and XCD-contiguous
// group numbering as pcdf; split tiles summed in group order by pcg_reduce_k (deterministic).
// bf16 (config 3): G staged as bf16 (the adjoint's bf16 output, or fp32 rounded), the fold sums in
// fp32 rounded once; weights = vfd_weight_fragments_bf16 mode 5; dx fp32 (K3's backward input).
#ifndef VFD_PG_BF_PF
#define VFD_PG_BF_PF 6      // bf16 B-fragment prefetch distance (steps; divides 18)
#endif
template <typename T>
struct PgCfg;
template <>
struct PgCfg<float> {
  static constexpr int OC = 16, XS = 20, STEPS = 4, PF = 4;   // o per atom, LDS elems / position, k-steps per tap
};
template <>
struct PgCfg<__bf16> {
  static constexpr int OC = 32, XS = 40, STEPS = 2, PF = VFD_PG_BF_PF;
};

constexpr int PG_PIX = 256;                     // interior pixels per tile (8 blocks of 32)
constexpr int PG_N = 128;                       // frustum channels per tile (4 waves x 32)
constexpr int PG_FRAG = PG_PIX * PG_N;          // floats of one tile's partial

struct PgGeom {
  int nbc, h, w, ntot, np, tpc, mtiles, ntn, ntile, och, natom, ngroup, hrows, cols, lds_elems;
};

__host__ __device__ inline int pg_lo(const PgGeom& g, int grp) {
  return (int)(((long long)grp * g.natom) / g.ngroup);
}

struct PgTile {
  int nt, bc, m0, y0;
};

// tile order: n-tile outermost (a group's consecutive tiles share the n-tile's weights)
__device__ __forceinline__ PgTile pg_tile(const PgGeom& g, int t) {
  PgTile r;
  const int mt = t % g.mtiles;
  r.nt = t / g.mtiles;
  r.bc = mt / g.tpc;
  r.m0 = (mt - r.bc * g.tpc) * PG_PIX;
  r.y0 = r.m0 / g.w;
  return r;
}

// 16-byte vectors of G: fp32 4 channels, bf16 8 channels; loads widen to fp32, the staging store
// rounds once to the LDS type
template <typename TG>
struct PgVec;
template <>
struct PgVec<float> {
  static constexpr int CH = 4;
  struct V { float x[4]; };
  static __device__ __forceinline__ V zero() { return V{{0.f, 0.f, 0.f, 0.f}}; }
  static __device__ __forceinline__ V load(const float* p) {
    const float4 f = *reinterpret_cast<const float4*>(p);
    return V{{f.x, f.y, f.z, f.w}};
  }
};
template <>
struct PgVec<__bf16> {
  static constexpr int CH = 8;
  struct V { float x[8]; };
  static __device__ __forceinline__ V zero() { return V{{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}}; }
  static __device__ __forceinline__ V load(const __bf16* p) {
    const bf16x8 b = *reinterpret_cast<const bf16x8*>(p);
    V v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v.x[j] = (float)b[j];
    return v;
  }
};

template <typename T, typename V, int CH>
__device__ __forceinline__ void pg_put(T* dst, const V& v) {
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int j = 0; j < CH; j += 4)
      *reinterpret_cast<float4*>(dst + j) = make_float4(v.x[j], v.x[j + 1], v.x[j + 2], v.x[j + 3]);
  } else {
#pragma unroll
    for (int j = 0; j < CH; j += 8) {
      bf16x8 b;
#pragma unroll
      for (int k = 0; k < 8; ++k) b[k] = (__bf16)v.x[j + k];
      *reinterpret_cast<bf16x8*>(dst + j) = b;
    }
  }
}

// loader waves (tid 0..255): staged rows 0 .. hrows-1 = G rows y0 - 1 .. (zero outside the camera),
// row hrows = F1 = G[2] + G[0], row hrows + 1 = F2 = G[h-3] + G[h-1] (each only when the tile holds
// pixel row 1 / h - 2); staged columns 0 .. w + 1 = G columns -1 .. w, w + 2 = E1 = G[.][2] + G[.][0],
// w + 3 = E2 = G[.][w-3] + G[.][w-1]; channels ch * OC .. + OC - 1.  A thread owns one (column,
// channel vector) and walks the rows: each staged element is the sum of <= 2 x 2 G vectors
// (rows ya / yb, columns xa / xb; -1 = absent), four rows' loads in flight.
template <typename T, typename TG>
__device__ __forceinline__ void pg_stage(const PgGeom& g, T* __restrict__ dst, const TG* __restrict__ gp, int atom,
                                         int tid) {
  typedef PgVec<TG> PV;
  constexpr int OC = PgCfg<T>::OC, XS = PgCfg<T>::XS, CH = PV::CH, QP = OC / CH, CPP = 256 / QP;
  const int t = atom / g.och, ch = atom - t * g.och;
  const PgTile tl = pg_tile(g, t);
  const int hw = g.h * g.w;
  const int ylast = ((tl.m0 + PG_PIX < hw ? tl.m0 + PG_PIX : hw) - 1) / g.w;
  const bool f1 = tl.y0 <= 1 && ylast >= 1, f2 = tl.y0 <= g.h - 2 && ylast >= g.h - 2;
  const int nrow = g.hrows + 2;
  const int q = tid % QP;
  const TG* src = gp + (size_t)tl.bc * hw * PC_O + ch * OC + CH * q;
  for (int c = tid / QP; c < g.cols; c += CPP) {
    int xa, xb = -1;
    if (c < g.w + 2) {
      xa = c - 1 < g.w ? c - 1 : -1;                 // -1 for c = 0 too
    } else if (c == g.w + 2) {
      xa = 2 < g.w ? 2 : -1;
      xb = 0;
    } else {
      xa = g.w - 3;
      xb = g.w - 1;
    }
    T* dcol = dst + c * XS + CH * q;
    for (int r0 = 0; r0 < nrow; r0 += 4) {
      typename PV::V v[4][4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = r0 + u;
        int ya = -1, yb = -1;
        if (r < g.hrows) {
          const int y = tl.y0 - 1 + r;
          ya = y >= 0 && y < g.h ? y : -1;
        } else if (r == g.hrows && f1) {
          ya = 2 < g.h ? 2 : -1;
          yb = 0;
        } else if (r == g.hrows + 1 && f2) {
          ya = g.h - 3;
          yb = g.h - 1;
        }
        const int ys[2] = {ya, yb}, xs[2] = {xa, xb};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int yy = ys[k >> 1], xx = xs[k & 1];
          v[u][k] = (r < nrow && yy >= 0 && xx >= 0) ? PV::load(src + ((size_t)yy * g.w + xx) * PC_O) : PV::zero();
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (r0 + u < nrow) {
          typename PV::V s = v[u][0];
#pragma unroll
          for (int j = 0; j < CH; ++j) s.x[j] = (s.x[j] + v[u][1].x[j]) + (v[u][2].x[j] + v[u][3].x[j]);
          pg_put<T, typename PV::V, CH>(dcol + (r0 + u) * g.cols * XS, s);
        }
      }
    }
  }
}

// fp32 weights: vfd_weight_fragments mode 2, float2 (s = 0, 1) at ((tap' * O/4 + oq) * np + n) * 2 + h;
// bf16: mode 5, bf16x8 at ((tap' * O/16 + q16) * np/32 + nb) * 64 + lane (o = 16 q16 + 8 h + j)
template <typename T, typename TG>
__global__ __launch_bounds__(PC_THREADS, 2) void pcg_main_k(PgGeom g, const TG* __restrict__ gp,
                                                           const void* __restrict__ Wd, float* __restrict__ dx,
                                                           float* __restrict__ partial) {
  constexpr int OC = PgCfg<T>::OC, XS = PgCfg<T>::XS, STEPS = PgCfg<T>::STEPS, PF = PgCfg<T>::PF;
  constexpr int ITERS = 9 * STEPS;
  constexpr bool BF = sizeof(T) == 2;
  typedef typename std::conditional<BF, bf16x8, float2>::type BFrag;
  typedef typename std::conditional<BF, bf16x8, float2>::type AFrag;
  extern __shared__ __attribute__((aligned(16))) unsigned char pg_raw[];
  T* lds = reinterpret_cast<T*>(pg_raw);
  const int grp = (g.ngroup % 8 == 0) ? (blockIdx.x % 8) * (g.ngroup / 8) + blockIdx.x / 8 : blockIdx.x;
  const int a_lo = pg_lo(g, grp), a_hi = pg_lo(g, grp + 1);
  if (a_lo >= a_hi) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool compute = wv < PC_WAVES;
  if (!compute) pg_stage<T, TG>(g, lds, gp, a_lo, threadIdx.x - 64 * PC_WAVES);
  __syncthreads();
  if (!compute) {
    for (int atom = a_lo; atom < a_hi; ++atom) {
      if (atom + 1 < a_hi)
        pg_stage<T, TG>(g, lds + ((atom + 1 - a_lo) & 1) * g.lds_elems, gp, atom + 1, threadIdx.x - 64 * PC_WAVES);
      __syncthreads();
    }
    return;
  }
  const int li = lane & 31, lh = lane >> 5;
  const int hw = g.h * g.w;
  f32x16 acc[8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[a][r] = 0.f;
  // B fragments: the lane's stream of atom a starts at bbase(a); iteration j = tap * STEPS + q adds
  // tap * tstride + q * qstride; prefetched PF iterations ahead (ITERS % PF == 0: static ring slots)
  static_assert(ITERS % PF == 0, "prefetch ring");
  const BFrag* wf = reinterpret_cast<const BFrag*>(Wd);
  const size_t qstride = BF ? (size_t)(g.np / 32) * 64 : (size_t)g.np * 2;
  const size_t tstride = (size_t)(BF ? PC_O / 16 : PC_O / 4) * qstride;
  auto bbase = [&](int atom) -> const BFrag* {
    const int t = atom / g.och, ch = atom - t * g.och;
    const int nt = t / g.mtiles;
    if constexpr (BF)
      return wf + (size_t)ch * STEPS * qstride + (size_t)(nt * (PG_N / 32) + wv) * 64 + lane;
    else
      return wf + (size_t)ch * STEPS * qstride + (size_t)(nt * PG_N + wv * 32 + li) * 2 + lh;
  };
  BFrag bq[PF];
  const BFrag* bcur = bbase(a_lo);
#pragma unroll
  for (int j = 0; j < PF; ++j) bq[j] = bcur[(j / STEPS) * tstride + (j % STEPS) * qstride];
  constexpr int LH = BF ? 8 : 2;                      // the lane half's element offset within a step
  for (int atom = a_lo; atom < a_hi; ++atom) {
    const int t = atom / g.och, ch = atom - t * g.och;
    const PgTile tl = pg_tile(g, t);
    const bool more = atom + 1 < a_hi;
    const BFrag* bnext = more ? bbase(atom + 1) : bcur;
    int pyx[8];                                       // (row << 16) | column of the lane's pixels
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      int m = tl.m0 + 32 * a + li;
      m = m < hw ? m : hw - 1;                        // pixels past the camera: computed, never stored
      const int y = m / g.w;
      pyx[a] = (y << 16) | (m - y * g.w);
    }
    const T* xb = lds + ((atom - a_lo) & 1) * g.lds_elems;
    auto offsets = [&](int tap, int* o1) {
      const int ky = tap / 3, kx = tap - 3 * ky;
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        const int px = pyx[a] & 0xFFFF, py = pyx[a] >> 16;
        const int col = (px == 1 && kx == 2) ? g.w + 2 : (px == g.w - 2 && kx == 0) ? g.w + 3 : px + kx;
        const int row = (py == 1 && ky == 2) ? g.hrows : (py == g.h - 2 && ky == 0) ? g.hrows + 1 : py - tl.y0 + ky;
        o1[a] = (row * g.cols + col) * XS + LH * lh;
      }
    };
    int o1c[8];
    offsets(0, o1c);
    AFrag afc[8], afn[8];
#pragma unroll
    for (int a = 0; a < 8; ++a) afc[a] = *reinterpret_cast<const AFrag*>(&xb[o1c[a]]);
#pragma unroll
    for (int j = 0; j < ITERS; ++j) {
      const int tap = j / STEPS, q = j % STEPS;
      const BFrag b = bq[j % PF];
      {                                               // refill the slot with iteration j + PF
        const int jn = j + PF;
        if (jn < ITERS)
          bq[j % PF] = bcur[(jn / STEPS) * tstride + (jn % STEPS) * qstride];
        else if (more)
          bq[j % PF] = bnext[((jn - ITERS) / STEPS) * tstride + ((jn - ITERS) % STEPS) * qstride];
      }
      if (q < STEPS - 1) {
#pragma unroll
        for (int a = 0; a < 8; ++a) afn[a] = *reinterpret_cast<const AFrag*>(&xb[o1c[a] + (OC / STEPS) * (q + 1)]);
      } else if (tap < 8) {                           // the current tap's loads are all issued
        offsets(tap + 1, o1c);
#pragma unroll
        for (int a = 0; a < 8; ++a) afn[a] = *reinterpret_cast<const AFrag*>(&xb[o1c[a]]);
      }
      if constexpr (BF) {
#pragma unroll
        for (int a = 0; a < 8; ++a) acc[a] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afc[a], b, acc[a], 0, 0, 0);
      } else {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int a = 0; a < 8; ++a)
            acc[a] = __builtin_amdgcn_mfma_f32_32x32x2f32(s2 ? afc[a].y : afc[a].x, s2 ? b.y : b.x, acc[a], 0, 0, 0);
      }
#pragma unroll
      for (int a = 0; a < 8; ++a) afc[a] = afn[a];
    }
    bcur = bnext;
    __syncthreads();                                  // buffer handed back to the loader waves
    if (ch == g.och - 1 || atom == a_hi - 1) {
      const int ts = t * g.och;
      const int n = tl.nt * PG_N + wv * 32 + li;
      if (ts >= a_lo && ts + g.och <= a_hi) {         // whole tile in this range: store
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = tl.m0 + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * lh;
            if (m < hw && n < g.ntot) {
              const int y = m / g.w, x = m - y * g.w;
              dx[(((size_t)tl.bc * (g.h + 2) + y + 1) * (g.w + 2) + x + 1) * g.ntot + n] = acc[a][r];
            }
            acc[a][r] = 0.f;
          }
      } else {                                        // split tile: partial slot
        const int slot = t == a_lo / g.och ? 0 : 1;
        float* dst = partial + ((size_t)grp * 2 + slot) * PG_FRAG + (size_t)wv * (PG_FRAG / PC_WAVES) + lane;
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            dst[(a * 16 + r) * 64] = acc[a][r];
            acc[a][r] = 0.f;
          }
      }
    }
  }
}

__global__ __launch_bounds__(256) void pcg_reduce_k(PgGeom g, const float* __restrict__ partial,
                                                    float* __restrict__ dx) {
  const int grp = blockIdx.x;
  const int lo = pg_lo(g, grp);
  if (grp == 0 || lo % g.och == 0) return;           // boundary on a tile edge: nothing split
  const int t = lo / g.och;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c0 = (grp - 1) * 2 + (t == pg_lo(g, grp - 1) / g.och ? 0 : 1), c1 = grp * 2;
  const PgTile tl = pg_tile(g, t);
  const int hw = g.h * g.w;
  constexpr int FPS = 8 * 16 / PC_FSL;
  constexpr int U = 4;
  const int contrib[2] = {c0, c1};
  const int n = tl.nt * PG_N + wv * 32 + (lane & 31);
  for (int fu = blockIdx.y * FPS; fu < (blockIdx.y + 1) * FPS; fu += U) {
    float su[U];
    frag_sums<U>(partial, contrib, 2, PG_FRAG, (size_t)wv * (PG_FRAG / PC_WAVES) + (fu * 64 + lane), su);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int f = fu + u;
      const int a = f >> 4, r = f & 15;
      const int m = tl.m0 + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (m < hw && n < g.ntot) {
        const int y = m / g.w, x = m - y * g.w;
        dx[(((size_t)tl.bc * (g.h + 2) + y + 1) * (g.w + 2) + x + 1) * g.ntot + n] = su[u];
      }
    }
  }
}

template <typename T>
static PgGeom pg_plan(const vfd_voxel_desc& d) {
  constexpr int OC = PgCfg<T>::OC, XS = PgCfg<T>::XS;
  PgGeom g;
  g.nbc = d.B * d.N;
  g.h = d.h;
  g.w = d.w;
  g.ntot = d.D * PC_CV;
  g.np = (g.ntot + 255) / 256 * 256;                  // the weight copies' n stride (mode 2 / 5)
  g.tpc = (d.h * d.w + PG_PIX - 1) / PG_PIX;
  g.mtiles = g.nbc * g.tpc;
  g.ntn = (g.ntot + PG_N - 1) / PG_N;
  g.ntile = g.ntn * g.mtiles;
  g.och = PC_O / OC;
  g.natom = g.ntile * g.och;
  int rows = d.w > 0 ? (PG_PIX - 1 + d.w - 1) / d.w + 1 : 1;   // pixel rows under 256 consecutive pixels
  rows = rows < d.h ? rows : d.h;
  g.hrows = rows + 2;
  g.cols = d.w + 4;
  g.lds_elems = (g.hrows + 2) * g.cols * XS;
  const int res = pc_resident();
  const int most = g.natom / g.och;
  g.ngroup = most < res ? (most > 0 ? most : 1) : res;
  return g;
}

template <typename T>
static bool pg_supported(const vfd_voxel_desc& d) {
  if (d.Cv != PC_CV || d.B <= 0 || d.N <= 0 || d.h < 2 || d.w < 2 || d.D <= 0 || d.D > 64) return false;
  if ((long long)d.h * d.w >= (1 << 16) * 256LL) return false;    // 16-bit row / column packing
  const PgGeom g = pg_plan<T>(d);
  return (size_t)2 * g.lds_elems * sizeof(T) <= PD_LDS_MAX;
}

// ---------------------------------------------------------------------------------------------
// bf16 folded data gradient on 2-D tiles ("pch", config 3): 16 x 16 interior pixels per tile, so an
// atom stages only the tile's 18 x 18 G halo (+ F1 / F2 rows and E1 / E2 columns when the tile holds
// pixel row / column 1 or h-2 / w-2): 400 positions per 256 pixels against pcg's whole rows (756 at
// w = 80) — at the bf16 MFMA rate pcg spends its time in the loader waves (timing without staging:
// 895 -> 458 us at config 2).  Pixel block a = tile rows 2a, 2a+1 (lane li: row 2a + li/16, column
// li%16).  LDS image [20 rows][RP][XS]: row pitch PH_RP elements = 448 dwords (a multiple of 64
// dwords), so the two tile rows of a pixel block fall into complementary bank slots for
// ds_read_b128 (positions 20 dwords apart within a row).  Same B fragments (mode 5), stream-K,
// prefetch ring, split-tile partials as pcg; ragged edge tiles (w or h not a multiple of 16) compute
// clamped pixels they never store.
constexpr int PH_T = 16;                        // tile side (pixels)
constexpr int PH_S = PH_T + 4;                  // staged rows / columns: 18 halo + the two fold slots
constexpr int PH_XS = 40;                       // bf16 per staged position (32 o + pad: 20 dwords)
constexpr int PH_RP = 896;                      // bf16 per staged row (448 dwords)
constexpr int PH_OC = 32;                       // o channels per atom
constexpr int PH_ELEMS = PH_S * PH_RP;          // bf16 per LDS buffer (35.8 KB)

struct PhGeom {
  int nbc, h, w, ntot, np, tpw, tpc, mtiles, ntile, och, natom, ngroup;
};

__host__ __device__ inline int ph_lo(const PhGeom& g, int grp) {
  return (int)(((long long)grp * g.natom) / g.ngroup);
}

struct PhTile {
  int nt, bc, y0, x0;
};

__device__ __forceinline__ PhTile ph_tile(const PhGeom& g, int t) {
  PhTile r;
  const int mt = t % g.mtiles;
  r.nt = t / g.mtiles;
  r.bc = mt / g.tpc;
  const int ti = mt - r.bc * g.tpc;
  r.y0 = (ti / g.tpw) * PH_T;
  r.x0 = (ti % g.tpw) * PH_T;
  return r;
}

// loader waves (tid 0..255): 400 positions x 4 eight-channel vectors, each the sum of <= 2 x 2 G
// vectors (rows ya / yb x columns xa / xb, -1 = absent); every load of a thread in flight together
constexpr int PH_PER = (PH_S * PH_S * 4 + 255) / 256;   // staged 16-B items per loader thread (7)
typedef bf16x8 PhRegs[PH_PER][4];

// loader waves (tid 0..255), phase 1: the atom's G rows (and fold partners) into registers
__device__ __forceinline__ void ph_fetch(const PhGeom& g, const __bf16* __restrict__ gp, int atom, int tid,
                                         PhRegs& v) {
  constexpr int NP = PH_S * PH_S, PER = PH_PER;
  const int t = atom / g.och, ch = atom - t * g.och;
  const PhTile tl = ph_tile(g, t);
  const bool f1 = tl.y0 == 0, f2 = tl.y0 <= g.h - 2 && tl.y0 + PH_T > g.h - 2;
  const bool e1 = tl.x0 == 0, e2 = tl.x0 <= g.w - 2 && tl.x0 + PH_T > g.w - 2;
  const int q = tid & 3;
  const __bf16* src = gp + (size_t)tl.bc * g.h * g.w * PC_O + ch * PH_OC + 8 * q;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int p = (tid >> 2) + 64 * k;
    const int r = p / PH_S, c = p - r * PH_S;
    int ya = -1, yb = -1, xa = -1, xb = -1;
    if (p < NP) {
      if (r < PH_T + 2) {
        const int y = tl.y0 - 1 + r;
        ya = y >= 0 && y < g.h ? y : -1;
      } else if (r == PH_T + 2 ? f1 : f2) {
        ya = r == PH_T + 2 ? (2 < g.h ? 2 : -1) : g.h - 3;
        yb = r == PH_T + 2 ? 0 : g.h - 1;
      }
      if (c < PH_T + 2) {
        const int x = tl.x0 - 1 + c;
        xa = x >= 0 && x < g.w ? x : -1;
      } else if (c == PH_T + 2 ? e1 : e2) {
        xa = c == PH_T + 2 ? (2 < g.w ? 2 : -1) : g.w - 3;
        xb = c == PH_T + 2 ? 0 : g.w - 1;
      }
    }
    const int ys[2] = {ya, yb}, xs[2] = {xa, xb};
    bf16x8 z;
#pragma unroll
    for (int e = 0; e < 8; ++e) z[e] = (__bf16)0.f;
    // only the two fold rows / columns have partners (yb / xb): the interior's 3 partner slots are
    // zero without a load or its address arithmetic
    v[k][0] = (ya >= 0 && xa >= 0) ? *reinterpret_cast<const bf16x8*>(src + ((size_t)ya * g.w + xa) * PC_O) : z;
    v[k][1] = v[k][2] = v[k][3] = z;
    if (yb >= 0 || xb >= 0) {
#pragma unroll
      for (int j = 1; j < 4; ++j) {
        const int yy = ys[j >> 1], xx = xs[j & 1];
        if (yy >= 0 && xx >= 0) v[k][j] = *reinterpret_cast<const bf16x8*>(src + ((size_t)yy * g.w + xx) * PC_O);
      }
    }
  }
}

// phase 2: the registers (fold partners summed) into one LDS image
__device__ __forceinline__ void ph_put(__bf16* __restrict__ dst, const PhRegs& v, int tid) {
  constexpr int NP = PH_S * PH_S, PER = PH_PER;
  const int q = tid & 3;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int p = (tid >> 2) + 64 * k;
    if (p < NP) {
      const int r = p / PH_S, c = p - r * PH_S;
      bf16x8 o = v[k][0];
      if (r >= PH_T + 2 || c >= PH_T + 2) {     // fold row / column: the partners' fp32 sum, rounded once
#pragma unroll
        for (int e = 0; e < 8; ++e)
          o[e] = (__bf16)(((float)v[k][0][e] + (float)v[k][1][e]) + ((float)v[k][2][e] + (float)v[k][3][e]));
      }
      *reinterpret_cast<bf16x8*>(dst + r * PH_RP + c * PH_XS + 8 * q) = o;
    }
  }
}


__device__ __forceinline__ void ph_stage(const PhGeom& g, __bf16* __restrict__ dst, const __bf16* __restrict__ gp,
                                         int atom, int tid) {
  PhRegs v;
  ph_fetch(g, gp, atom, tid, v);
  ph_put(dst, v, tid);
}

__global__ __launch_bounds__(PC_THREADS, 2) void pch_main_k(PhGeom g, const __bf16* __restrict__ gp,
                                                           const bf16x8* __restrict__ Wd, float* __restrict__ dx,
                                                           float* __restrict__ partial) {
  constexpr int STEPS = PH_OC / 16, PF = VFD_PG_BF_PF, ITERS = 9 * STEPS;
  static_assert(ITERS % PF == 0, "prefetch ring");
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * PH_ELEMS];
  const int grp = (g.ngroup % 8 == 0) ? (blockIdx.x % 8) * (g.ngroup / 8) + blockIdx.x / 8 : blockIdx.x;
  const int a_lo = ph_lo(g, grp), a_hi = ph_lo(g, grp + 1);
  if (a_lo >= a_hi) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool compute = wv < PC_WAVES;
#if VFD_PH_PIPE
  // loader waves two atoms ahead: the rows of atom k + 2 are fetched into registers right after
  // atom k + 1's are put in LDS, so their L2 / MALL round trip overlaps a whole atom of MFMAs and
  // the barrier (one atom ahead, the round trip was exposed on every atom: 0.23 of 0.91 ms)
  PhRegs pv;
  const int ltid = threadIdx.x - 64 * PC_WAVES;
  if (!compute) {
    ph_fetch(g, gp, a_lo, ltid, pv);
    ph_put(lds, pv, ltid);
    if (a_lo + 1 < a_hi) ph_fetch(g, gp, a_lo + 1, ltid, pv);
  }
  __syncthreads();
  if (!compute) {
    for (int atom = a_lo; atom < a_hi; ++atom) {
      if (atom + 1 < a_hi) {
        ph_put(lds + ((atom + 1 - a_lo) & 1) * PH_ELEMS, pv, ltid);
        if (atom + 2 < a_hi) ph_fetch(g, gp, atom + 2, ltid, pv);
      }
      __syncthreads();
    }
    return;
  }
#else
  if (!compute) ph_stage(g, lds, gp, a_lo, threadIdx.x - 64 * PC_WAVES);
  __syncthreads();
  if (!compute) {
    for (int atom = a_lo; atom < a_hi; ++atom) {
      if (atom + 1 < a_hi) ph_stage(g, lds + ((atom + 1 - a_lo) & 1) * PH_ELEMS, gp, atom + 1, threadIdx.x - 64 * PC_WAVES);
      __syncthreads();
    }
    return;
  }
#endif
  const int li = lane & 31, lh = lane >> 5;
  f32x16 acc[8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[a][r] = 0.f;
  const size_t qstride = (size_t)(g.np / 32) * 64, tstride = (size_t)(PC_O / 16) * qstride;
  auto bbase = [&](int atom) -> const bf16x8* {
    const int t = atom / g.och, ch = atom - t * g.och;
    const int nt = t / g.mtiles;
    return Wd + (size_t)ch * STEPS * qstride + (size_t)(nt * (PG_N / 32) + wv) * 64 + lane;
  };
  bf16x8 bq[PF];
  const bf16x8* bcur = bbase(a_lo);
#pragma unroll
  for (int j = 0; j < PF; ++j) bq[j] = bcur[(j / STEPS) * tstride + (j % STEPS) * qstride];
  const int ly = li >> 4, lx = li & 15;
  for (int atom = a_lo; atom < a_hi; ++atom) {
    const int t = atom / g.och, ch = atom - t * g.och;
    const PhTile tl = ph_tile(g, t);
    const bool more = atom + 1 < a_hi;
    const bf16x8* bnext = more ? bbase(atom + 1) : bcur;
    // the lane's pixel column (clamped into the camera) and, per block, its row
    const int px = min(tl.x0 + lx, g.w - 1);
    int py[8];
#pragma unroll
    for (int a = 0; a < 8; ++a) py[a] = min(tl.y0 + 2 * a + ly, g.h - 1);
    const __bf16* xb = lds + ((atom - a_lo) & 1) * PH_ELEMS;
    auto offsets = [&](int tap, int* o1) {
      const int ky = tap / 3, kx = tap - 3 * ky;
      const int col = (px == 1 && kx == 2) ? PH_T + 2 : (px == g.w - 2 && kx == 0) ? PH_T + 3 : px - tl.x0 + kx;
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        const int row = (py[a] == 1 && ky == 2) ? PH_T + 2 : (py[a] == g.h - 2 && ky == 0) ? PH_T + 3 : py[a] - tl.y0 + ky;
        o1[a] = row * PH_RP + col * PH_XS + 8 * lh;
      }
    };
    int o1c[8];
    offsets(0, o1c);
    bf16x8 afc[8], afn[8];
#pragma unroll
    for (int a = 0; a < 8; ++a) afc[a] = *reinterpret_cast<const bf16x8*>(&xb[o1c[a]]);
#pragma unroll
    for (int j = 0; j < ITERS; ++j) {
      const int tap = j / STEPS, q = j % STEPS;
      const bf16x8 b = bq[j % PF];
      {
        const int jn = j + PF;
        if (jn < ITERS)
          bq[j % PF] = bcur[(jn / STEPS) * tstride + (jn % STEPS) * qstride];
        else if (more)
          bq[j % PF] = bnext[((jn - ITERS) / STEPS) * tstride + ((jn - ITERS) % STEPS) * qstride];
      }
      if (q < STEPS - 1) {
#pragma unroll
        for (int a = 0; a < 8; ++a) afn[a] = *reinterpret_cast<const bf16x8*>(&xb[o1c[a] + 16 * (q + 1)]);
      } else if (tap < 8) {
        offsets(tap + 1, o1c);
#pragma unroll
        for (int a = 0; a < 8; ++a) afn[a] = *reinterpret_cast<const bf16x8*>(&xb[o1c[a]]);
      }
#pragma unroll
      for (int a = 0; a < 8; ++a) acc[a] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afc[a], b, acc[a], 0, 0, 0);
#pragma unroll
      for (int a = 0; a < 8; ++a) afc[a] = afn[a];
    }
    bcur = bnext;
    __syncthreads();                                  // buffer handed back to the loader waves
    if (ch == g.och - 1 || atom == a_hi - 1) {
      const int ts = t * g.och;
      const int n = tl.nt * PG_N + wv * 32 + li;
      if (ts >= a_lo && ts + g.och <= a_hi) {         // whole tile in this range: store
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rr = (r & 3) + 8 * (r >> 2) + 4 * lh;       // pixel of block a: tile row 2a + rr/16
            const int y = tl.y0 + 2 * a + (rr >> 4), x = tl.x0 + (rr & 15);
            if (y < g.h && x < g.w && n < g.ntot)
              dx[(((size_t)tl.bc * (g.h + 2) + y + 1) * (g.w + 2) + x + 1) * g.ntot + n] = acc[a][r];
            acc[a][r] = 0.f;
          }
      } else {
        const int slot = t == a_lo / g.och ? 0 : 1;
        float* dst = partial + ((size_t)grp * 2 + slot) * PG_FRAG + (size_t)wv * (PG_FRAG / PC_WAVES) + lane;
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            dst[(a * 16 + r) * 64] = acc[a][r];
            acc[a][r] = 0.f;
          }
      }
    }
  }
}

__global__ __launch_bounds__(256) void pch_reduce_k(PhGeom g, const float* __restrict__ partial,
                                                    float* __restrict__ dx) {
  const int grp = blockIdx.x;
  const int lo = ph_lo(g, grp);
  if (grp == 0 || lo % g.och == 0) return;
  const int t = lo / g.och;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c0 = (grp - 1) * 2 + (t == ph_lo(g, grp - 1) / g.och ? 0 : 1), c1 = grp * 2;
  const PhTile tl = ph_tile(g, t);
  constexpr int FPS = 8 * 16 / PC_FSL;
  constexpr int U = 4;
  const int contrib[2] = {c0, c1};
  const int n = tl.nt * PG_N + wv * 32 + (lane & 31);
  for (int fu = blockIdx.y * FPS; fu < (blockIdx.y + 1) * FPS; fu += U) {
    float su[U];
    frag_sums<U>(partial, contrib, 2, PG_FRAG, (size_t)wv * (PG_FRAG / PC_WAVES) + (fu * 64 + lane), su);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int f = fu + u;
      const int a = f >> 4, r = f & 15;
      const int rr = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const int y = tl.y0 + 2 * a + (rr >> 4), x = tl.x0 + (rr & 15);
      if (y < g.h && x < g.w && n < g.ntot)
        dx[(((size_t)tl.bc * (g.h + 2) + y + 1) * (g.w + 2) + x + 1) * g.ntot + n] = su[u];
    }
  }
}

static PhGeom ph_plan(const vfd_voxel_desc& d) {
  PhGeom g;
  g.nbc = d.B * d.N;
  g.h = d.h;
  g.w = d.w;
  g.ntot = d.D * PC_CV;
  g.np = (g.ntot + 255) / 256 * 256;
  g.tpw = (d.w + PH_T - 1) / PH_T;
  g.tpc = ((d.h + PH_T - 1) / PH_T) * g.tpw;
  g.mtiles = g.nbc * g.tpc;
  g.ntile = ((g.ntot + PG_N - 1) / PG_N) * g.mtiles;
  g.och = PC_O / PH_OC;
  g.natom = g.ntile * g.och;
  const int res = pc_resident();
  const int most = g.natom / g.och;
  g.ngroup = most < res ? (most > 0 ? most : 1) : res;
  return g;
}

static bool ph_supported(const vfd_voxel_desc& d) {
  return d.Cv == PC_CV && d.B > 0 && d.N > 0 && d.h >= 2 && d.w >= 2 && d.D > 0 && d.D <= 64 &&
         (long long)d.B * d.N * d.h * d.w < (1LL << 31) / 256;
}

// =============================================================================================
// K3C weight gradient — reduce_dim's first conv, d weight and d bias (volumetric_fusionnet.py:59-60,
// 265 backward), as an fp32 MFMA GEMM over the pixels of all cameras:
//
//   dW[o, n, ky, kx] = sum_{bc, y, x} G[bc, y, x, o] * Xp[bc, y + ky, x + kx, n],   db[o] = sum G
//
// G = d pre-activation [B*N, h, w, O] (NHWC), Xp = the frustum features K3C's forward wrote as its
// side output [B*N, h+2, w+2, D*Cv] (n = d*Cv + c).  M = the 256 output channels, N = 32 frustum
// channels x 9 taps, K = pixels: an output tile (one 32-channel block of n) is 8 x 9 MFMA blocks;
// wave w of the 8 owns o-block w and all 9 taps (9 f32x16 accumulators), so one A fragment (G)
// feeds 9 MFMAs whose B fragments are the 9 tap-shifted X positions of the same LDS halo.  All 8
// waves compute (two per SIMD, so one wave's LDS waits are covered by the other's MFMAs) and all
// stage: an atom = (tile, camera, 2 x 16 pixel tile); during atom a each thread's global loads of
// atom a+1 (its share of 32 G rows x 256 o and the 4 x 18 x 32 Xp halo) are in flight, and land
// in the other half of a double-buffered LDS image after the wave's MFMAs (one barrier per atom).
// Stream-K over the atoms (one workgroup per CU, contiguous equal ranges, tile-major): every tile
// a range meets leaves a partial in MFMA fragment order; `pcw_reduce_k` sums a tile's partials in
// workgroup order (deterministic) and writes dW straight into the reference layout
// [O, Cv*D (c*D + d), 3, 3].
constexpr int PW_WAVES = 8;
constexpr int PW_NT = 32;                       // frustum channels per tile
constexpr int PW_TR = 2, PW_TC = 16;            // pixel tile of an atom
constexpr int PW_PIX = PW_TR * PW_TC;
constexpr int PW_HR = PW_TR + 2, PW_HC = PW_TC + 2;
constexpr int PW_NPOS = PW_HR * PW_HC;          // 72 halo positions
constexpr int PW_GS = PC_O + 32;                // LDS floats per staged G pixel (lane halves on other banks)
constexpr int PW_XS = PW_NT;                    // LDS floats per staged X position
constexpr int PW_BUF = PW_PIX * PW_GS + PW_NPOS * PW_XS;
constexpr int PW_FRAG = PW_WAVES * 9 * 16 * 64;  // floats of one tile's partial
constexpr int PW_GV = PW_PIX * PC_O / 4 / PC_THREADS;                    // 4 float4 of G per thread
constexpr int PW_XV = (PW_NPOS * PW_XS / 4 + PC_THREADS - 1) / PC_THREADS;  // 2 float4 of Xp per thread

struct PwGeom {
  int nbc, h, w, ntot, D, tc, tiles_img, L, ntile, natom, ngroup, slots;
};

__host__ __device__ inline long long pw_lo(const PwGeom& g, int grp) {
  return ((long long)grp * g.natom) / g.ngroup;
}

struct PwStage {
  float4 gv[PW_GV], xv[PW_XV];
};

// a thread's share of atom `atom`: G rows of its 32 pixels and the Xp halo, into registers
__device__ __forceinline__ void pw_fetch(const PwGeom& g, PwStage& st, const float* __restrict__ gp,
                                         const float* __restrict__ xp, int atom, int tid) {
  const int t = atom / g.L, within = atom - t * g.L;
  const int bc = within / g.tiles_img, ti = within - bc * g.tiles_img;
  const int y0 = (ti / g.tc) * PW_TR, x0 = (ti % g.tc) * PW_TC;
  const int wo = g.w + 2;
#pragma unroll
  for (int u = 0; u < PW_GV; ++u) {
    const int e = tid + PC_THREADS * u, px = e >> 6, q = e & 63;
    const int y = y0 + (px >> 4), x = x0 + (px & 15);
    st.gv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (y < g.h && x < g.w)
      st.gv[u] = *reinterpret_cast<const float4*>(gp + (((size_t)bc * g.h + y) * g.w + x) * PC_O + 4 * q);
  }
#pragma unroll
  for (int u = 0; u < PW_XV; ++u) {
    const int e = tid + PC_THREADS * u, pos = e >> 3, q = e & 7;
    const int r = pos / PW_HC, c = pos - r * PW_HC;
    const int Y = y0 + r, X = x0 + c;
    st.xv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (pos < PW_NPOS && Y < g.h + 2 && X < wo)
      st.xv[u] = *reinterpret_cast<const float4*>(xp + (((size_t)bc * (g.h + 2) + Y) * wo + X) * g.ntot + t * PW_NT + 4 * q);
  }
}

__device__ __forceinline__ void pw_put(const PwStage& st, float* __restrict__ dst, int tid) {
#pragma unroll
  for (int u = 0; u < PW_GV; ++u) {
    const int e = tid + PC_THREADS * u, px = e >> 6, q = e & 63;
    *reinterpret_cast<float4*>(dst + px * PW_GS + 4 * q) = st.gv[u];
  }
  float* xd = dst + PW_PIX * PW_GS;
#pragma unroll
  for (int u = 0; u < PW_XV; ++u) {
    const int e = tid + PC_THREADS * u, pos = e >> 3, q = e & 7;
    if (pos < PW_NPOS) *reinterpret_cast<float4*>(xd + pos * PW_XS + 4 * q) = st.xv[u];
  }
}

__global__ __launch_bounds__(PC_THREADS, 2) void pcw_main_k(PwGeom g, const float* __restrict__ gp,
                                                           const float* __restrict__ xp,
                                                           float* __restrict__ partial) {
  __shared__ float lds[2][PW_BUF];
  const int grp = blockIdx.x;
  const int a_lo = (int)pw_lo(g, grp), a_hi = (int)pw_lo(g, grp + 1);
  if (a_lo >= a_hi) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int li = lane & 31, kk = lane >> 5;
  {
    PwStage st;
    pw_fetch(g, st, gp, xp, a_lo, tid);
    pw_put(st, lds[0], tid);
  }
  __syncthreads();
  f32x16 acc[9];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[k][r] = 0.f;
  const int first_tile = a_lo / g.L;
  int tile = first_tile;
  auto flush = [&](int tl) {
    float* dst = partial + (((size_t)grp * g.slots + (tl - first_tile)) * PW_WAVES + wv) * (9 * 16 * 64) + lane;
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        dst[(k * 16 + r) * 64] = acc[k][r];
        acc[k][r] = 0.f;
      }
  };
  for (int atom = a_lo; atom < a_hi; ++atom) {
    const int t = atom / g.L;
    if (t != tile) {
      flush(tile);
      tile = t;
    }
    PwStage st;
    const bool more = atom + 1 < a_hi;
    if (more) pw_fetch(g, st, gp, xp, atom + 1, tid);        // in flight during this atom's MFMAs
    const float* gb = lds[(atom - a_lo) & 1] + kk * PW_GS + 32 * wv + li;       // lane's G column
    const float* xb = lds[(atom - a_lo) & 1] + PW_PIX * PW_GS + kk * PW_XS + li;  // lane's X column
    // pixel pair s: pixels 2s (lanes 0-31) and 2s+1 (lanes 32-63), one tile row
#pragma unroll
    for (int s = 0; s < PW_PIX / 2; ++s) {
      const int p = 2 * s, py = p >> 4, px = p & 15;
      const float a = gb[p * PW_GS];
#pragma unroll
      for (int k = 0; k < 9; ++k)
        acc[k] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, xb[((py + k / 3) * PW_HC + px + (k % 3)) * PW_XS], acc[k],
                                                      0, 0, 0);
    }
    if (more) pw_put(st, lds[(atom + 1 - a_lo) & 1], tid);
    __syncthreads();
  }
  flush(tile);
}

// the workgroup whose range holds atom a
__device__ __forceinline__ int pw_owner(const PwGeom& g, long long a) {
  int grp = (int)((a * g.ngroup) / g.natom);
  while (grp + 1 < g.ngroup && pw_lo(g, grp + 1) <= a) ++grp;
  while (grp > 0 && pw_lo(g, grp) > a) --grp;
  return grp;
}

// Workgroup (o quad, c half, chunk of PW_DC depth bins): the partials of the chunk's tiles (tile =
// 32-channel block n / 32 = 2d + c half) for the quad's 4 output channels, summed in workgroup
// order into LDS (128-B runs of the fragments), then written as dW[o][c*D + d][tap]: runs of
// PW_DC * 9 consecutive floats per (o, c), whole cache lines instead of 36-B pieces.
constexpr int PW_DC = 10;

constexpr int PW_MAXC = 16;     // contributors of one tile the reduce handles (host-checked)

__global__ __launch_bounds__(256) void pcw_reduce_k(PwGeom g, const float* __restrict__ partial,
                                                    float* __restrict__ dw) {
  __shared__ float sm[PW_DC * 4 * 32 * 9];
  __shared__ long long off[PW_DC][PW_MAXC];
  __shared__ int ncon[PW_DC];
  const int oq = blockIdx.x, ch = blockIdx.y & 1, d0 = (blockIdx.y >> 1) * PW_DC;
  const int nd = g.D - d0 < PW_DC ? g.D - d0 : PW_DC;
  const int wb = oq >> 3, lh = oq & 1, rb = ((oq & 7) >> 1) * 4;
  if (threadIdx.x < nd) {          // the chunk's tiles: contributing workgroups, in order
    const int dl = threadIdx.x, t = 2 * (d0 + dl) + ch;
    const int g0 = pw_owner(g, (long long)t * g.L), g1 = pw_owner(g, (long long)(t + 1) * g.L - 1);
    ncon[dl] = g1 - g0 + 1;
    for (int grp = g0; grp <= g1; ++grp) {
      const int slot = t - (int)(pw_lo(g, grp) / g.L);
      off[dl][grp - g0] = (((long long)grp * g.slots + slot) * PW_WAVES + wb) * (9 * 16 * 64);
    }
  }
  __syncthreads();
  // 4 elements per thread per pass, every contributor load of the 4 in flight before the sums
  // (contributors beyond the fourth: a plain loop; they occur only for very short ranges)
  constexpr int U = 4;
  const int total = nd * 4 * 32 * 9;
  for (int e0 = threadIdx.x; e0 < total; e0 += 256 * U) {
    float a[U][4];
    int fo[U], dls[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + 256 * u;
      const int ee = e < total ? e : total - 1;
      const int cl = ee & 31, ol = (ee >> 5) & 3, tap = (ee >> 7) % 9, dl = ee / (4 * 32 * 9);
      fo[u] = (tap * 16 + rb + ol) * 64 + cl + 32 * lh;
      dls[u] = dl;
#pragma unroll
      for (int k = 0; k < 4; ++k) a[u][k] = k < ncon[dl] ? partial[off[dl][k] + fo[u]] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + 256 * u;
      if (e >= total) break;
      float v = ((a[u][0] + a[u][1]) + a[u][2]) + a[u][3];
      for (int k = 4; k < ncon[dls[u]]; ++k) v += partial[off[dls[u]][k] + fo[u]];
      const int cl = e & 31, ol = (e >> 5) & 3, tap = (e >> 7) % 9;
      sm[((dls[u] * 4 + ol) * 32 + cl) * 9 + tap] = v;
    }
  }
  __syncthreads();
  const int run = nd * 9;
  for (int e = threadIdx.x; e < 4 * 32 * run; e += 256) {
    const int k = e % run, oc = e / run, cl = oc & 31, ol = oc >> 5;
    const int dl = k / 9, tap = k - dl * 9;
    const int o = 4 * oq + ol, c = 32 * ch + cl;
    dw[((size_t)o * g.ntot + c * g.D + d0) * 9 + k] = sm[((dl * 4 + ol) * 32 + cl) * 9 + tap];
  }
}

// d bias: fixed-order column sums of G — blocks of PW_BIAS_ROWS rows, then the block partials
constexpr int PW_BIAS_ROWS = 64;

__global__ __launch_bounds__(256) void pcw_bias_k(int rows, const float* __restrict__ gp, float* __restrict__ part) {
  const int r0 = blockIdx.x * PW_BIAS_ROWS;
  const int r1 = r0 + PW_BIAS_ROWS < rows ? r0 + PW_BIAS_ROWS : rows;
  float s = 0.f;
  for (int r = r0; r < r1; r += 8) {            // 8 rows in flight, summed in row order
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = r + k < r1 ? gp[(size_t)(r + k) * PC_O + threadIdx.x] : 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k];
  }
  part[blockIdx.x * PC_O + threadIdx.x] = s;
}

// workgroup = 4 channels x 64 lanes: lane j sums partial rows j, j + 64, ... of its channel, then
// the 64 lane sums are added in lane order
__global__ __launch_bounds__(256) void pcw_bias_fin_k(int nblk, const float* __restrict__ part, float* __restrict__ db) {
  __shared__ float sh[4][64];
  const int c = 4 * blockIdx.x + (threadIdx.x & 3), j = threadIdx.x >> 2;
  float s = 0.f;
  for (int b = j; b < nblk; b += 64) s += part[b * PC_O + c];
  sh[threadIdx.x & 3][j] = s;
  __syncthreads();
  if (threadIdx.x < 4) {
    float t = 0.f;
    for (int k = 0; k < 64; ++k) t += sh[threadIdx.x][k];
    db[4 * blockIdx.x + threadIdx.x] = t;
  }
}

static PwGeom pw_plan(const vfd_voxel_desc& d) {
  PwGeom g;
  g.nbc = d.B * d.N;
  g.h = d.h;
  g.w = d.w;
  g.D = d.D;
  g.ntot = d.D * PC_CV;
  g.tc = (d.w + PW_TC - 1) / PW_TC;
  g.tiles_img = ((d.h + PW_TR - 1) / PW_TR) * g.tc;
  g.L = g.nbc * g.tiles_img;
  g.ntile = g.ntot / PW_NT;
  g.natom = g.ntile * g.L;
  const int res = pc_resident();
  g.ngroup = g.natom < res ? g.natom : res;
  const long long range = (g.natom + g.ngroup - 1) / g.ngroup;
  g.slots = (int)((range - 1) / g.L) + 2;
  return g;
}

static bool pw_supported(const vfd_voxel_desc& d) {
  if (!(d.Cv == PC_CV && d.B > 0 && d.N > 0 && d.h >= 1 && d.w >= 1 && d.D > 0 && d.D <= 64)) return false;
  const PwGeom g = pw_plan(d);
  const long long range = g.natom / g.ngroup;           // shortest range
  return range > 0 && (g.L + range - 1) / range + 1 <= PW_MAXC;   // workgroups meeting one tile
}

// =============================================================================================
// bf16 weight / bias gradient of a 3x3 conv (stride 1 or 2) on MFMA — K3C's reduce_dim[0] (stride 1,
// the bf16 frustum side output) and K2C's pose reduce_dim[0] (stride 2, the fp32 BEV map rounded to
// bf16 as it is staged) under config 3's autocast (volumetric_fusionnet.py:59-60, 105-114, 265,
// 338-343 backward; MIOpen's bf16 weight gradient before):
//
//   dW[o, n, ky, kx] = sum_{img, y, x} G[img, y, x, o] * X[img, s y + ky, s x + kx, n]
//
// M = the 256 output channels (8 waves x one 32-channel block), N = 32 input channels x 9 taps per
// tile (9 accumulators per wave), K = pixels, 16 per v_mfma_f32_32x32x16_bf16.  An atom = (tile,
// image, 4 x 16 output pixels): the G rows (64 pixels x 256 o) and the X halo ((3s + 3) x (15s + 3)
// positions x 32 n) staged in LDS in their natural [pixel][channel] layouts and read as MFMA operands
// with ds_read_b64_tr_b16 (the transpose read delivers 4 consecutive pixels of one channel per lane;
// a tap is only a different per-lane row address, so no shifted copies).  G rows padded to 576 B and X
// positions at 64 B make both transposed reads conflict-free for stride 1.  Every wave stages its share
// of the next atom into registers during the current atom's MFMAs (as pcw_main_k).  Stream-K over atoms;
// partials in pcw_main_k's fragment layout (pcw_reduce_k sums them for K3C in the reference channel order;
// pwb_reduce_map_k in the map's order for K2C, then the pose weight swap).
constexpr int WB_TR = 4, WB_TC = 16, WB_PIX = WB_TR * WB_TC;
constexpr int WB_GP = 288;                      // bf16 per staged G pixel (256 o + pad: 576 B)
constexpr int WB_XP = 32;                       // bf16 per staged X position (64 B)
constexpr int WB_XMAX = (3 * 2 + 3) * (15 * 2 + 3);   // halo positions at stride 2 (297)
constexpr int WB_BUF = WB_PIX * WB_GP + WB_XMAX * WB_XP;   // bf16 per buffer (55.9 KB)

struct WbGeom {
  int nimg, ho, wo, hp, wp, s, C, tc, tiles_img, L, ntile, natom, ngroup, slots, hr, hc;
};

__host__ __device__ inline long long wb_lo(const WbGeom& g, int grp) { return ((long long)grp * g.natom) / g.ngroup; }

typedef short wb_s4 __attribute__((ext_vector_type(4)));

// X vectors: XV channels of TX per load — 8 bf16 (16 B) or 4 fp32 (16 B, rounded when put), or
// 4 bf16 (8 B) for the bf16 BEV map of K2C (C = 5140: a multiple of 4, not of 8)
template <typename TX, int XV>
struct WbXVec {
  typedef typename std::conditional<sizeof(TX) == 2, typename std::conditional<XV == 8, uint4, uint2>::type,
                                    float4>::type type;
};

template <typename TX, int XV>
struct WbStage {
  uint4 gv[WB_PIX * PC_O / 8 / PC_THREADS];                         // 4 x 8 bf16 of G
  typename WbXVec<TX, XV>::type xv[(WB_XMAX * WB_XP / XV + PC_THREADS - 1) / PC_THREADS];
};

template <typename TX, int XV>
__device__ __forceinline__ void wb_fetch(const WbGeom& g, WbStage<TX, XV>& st, const __bf16* __restrict__ gp,
                                         const TX* __restrict__ xp, int atom, int tid) {
  constexpr int NXV = sizeof(st.xv) / sizeof(st.xv[0]);
  typedef typename WbXVec<TX, XV>::type XT;
  const int t = atom / g.L, within = atom - t * g.L;
  const int img = within / g.tiles_img, ti = within - img * g.tiles_img;
  const int y0 = (ti / g.tc) * WB_TR, x0 = (ti % g.tc) * WB_TC;
#pragma unroll
  for (int u = 0; u < (int)(sizeof(st.gv) / sizeof(st.gv[0])); ++u) {
    const int e = tid + PC_THREADS * u, px = e >> 5, q = e & 31;     // 32 vectors of 8 o per pixel
    const int y = y0 + (px >> 4), x = x0 + (px & 15);
    st.gv[u] = make_uint4(0u, 0u, 0u, 0u);
    if (y < g.ho && x < g.wo)
      st.gv[u] = *reinterpret_cast<const uint4*>(gp + (((size_t)img * g.ho + y) * g.wo + x) * PC_O + 8 * q);
  }
  const int npos = g.hr * g.hc, vpp = WB_XP / XV;
#pragma unroll
  for (int u = 0; u < NXV; ++u) {
    const int e = tid + PC_THREADS * u, pos = e / vpp, q = e - pos * vpp;
    const int r = pos / g.hc, c = pos - r * g.hc;
    const int Y = g.s * y0 + r, X = g.s * x0 + c, n = t * 32 + XV * q;
    memset(&st.xv[u], 0, sizeof(st.xv[u]));
    if (pos < npos && Y < g.hp && X < g.wp && n < g.C)
      st.xv[u] = *reinterpret_cast<const XT*>(xp + (((size_t)img * g.hp + Y) * g.wp + X) * g.C + n);
  }
}

template <typename TX, int XV>
__device__ __forceinline__ void wb_put(const WbGeom& g, const WbStage<TX, XV>& st, __bf16* __restrict__ dst, int tid) {
  constexpr int NXV = sizeof(st.xv) / sizeof(st.xv[0]);
  typedef typename WbXVec<TX, XV>::type XT;
#pragma unroll
  for (int u = 0; u < (int)(sizeof(st.gv) / sizeof(st.gv[0])); ++u) {
    const int e = tid + PC_THREADS * u, px = e >> 5, q = e & 31;
    *reinterpret_cast<uint4*>(dst + px * WB_GP + 8 * q) = st.gv[u];
  }
  __bf16* xd = dst + WB_PIX * WB_GP;
  const int npos = g.hr * g.hc, vpp = WB_XP / XV;
#pragma unroll
  for (int u = 0; u < NXV; ++u) {
    const int e = tid + PC_THREADS * u, pos = e / vpp, q = e - pos * vpp;
    if (pos < npos) {
      if constexpr (sizeof(TX) == 2) {
        *reinterpret_cast<XT*>(xd + pos * WB_XP + XV * q) = st.xv[u];
      } else {
        bf16x4 b;
        b[0] = (__bf16)st.xv[u].x;
        b[1] = (__bf16)st.xv[u].y;
        b[2] = (__bf16)st.xv[u].z;
        b[3] = (__bf16)st.xv[u].w;
        *reinterpret_cast<bf16x4*>(xd + pos * WB_XP + XV * q) = b;
      }
    }
  }
}

__device__ __forceinline__ bf16x8 wb_tr8(const __bf16* p0, const __bf16* p1) {
  typedef __attribute__((address_space(3))) wb_s4 lds_s4;
  const wb_s4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p0));
  const wb_s4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p1));
  bf16x8 r;
  __builtin_memcpy(&r, &a, 8);
  __builtin_memcpy(reinterpret_cast<char*>(&r) + 8, &b, 8);
  return r;
}

template <typename TX, int XV = 16 / sizeof(TX)>
__global__ __launch_bounds__(PC_THREADS, 2) void pwb_main_k(WbGeom g, const __bf16* __restrict__ gp,
                                                           const TX* __restrict__ xp, float* __restrict__ partial) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * WB_BUF];
  const int grp = blockIdx.x;
  const int a_lo = (int)wb_lo(g, grp), a_hi = (int)wb_lo(g, grp + 1);
  if (a_lo >= a_hi) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  {
    WbStage<TX, XV> st;
    wb_fetch<TX, XV>(g, st, gp, xp, a_lo, tid);
    wb_put<TX, XV>(g, st, lds, tid);
  }
  __syncthreads();
  f32x16 acc[9];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[k][r] = 0.f;
  const int first_tile = a_lo / g.L;
  int tile = first_tile;
  auto flush = [&](int tl) {
    float* dst = partial + (((size_t)grp * g.slots + (tl - first_tile)) * PW_WAVES + wv) * (9 * 16 * 64) + lane;
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        dst[(k * 16 + r) * 64] = acc[k][r];
        acc[k][r] = 0.f;
      }
  };
  // transposed-read lane roles: group gq = lane >> 4 (column half gq & 1, row half gq >> 1); within
  // the group lane 4q + p supplies row q, columns 4p .. 4p + 3
  const int gq = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int colh = 16 * (gq & 1) + 4 * p, rowh = 8 * (gq >> 1) + q;
  for (int atom = a_lo; atom < a_hi; ++atom) {
    const int t = atom / g.L;
    if (t != tile) {
      flush(tile);
      tile = t;
    }
    WbStage<TX, XV> st;
    const bool more = atom + 1 < a_hi;
    if (more) wb_fetch<TX, XV>(g, st, gp, xp, atom + 1, tid);           // in flight during this atom's MFMAs
    const __bf16* gb = lds + ((atom - a_lo) & 1) * WB_BUF;
    const __bf16* xb = gb + WB_PIX * WB_GP;
#pragma unroll 1
    for (int ks = 0; ks < WB_TR; ++ks) {
      // A = G^T: rows = pixels 16 ks + rowh (+4), columns = this wave's o block
      const __bf16* ga = gb + (16 * ks + rowh) * WB_GP + 32 * wv + colh;
      const bf16x8 a = wb_tr8(ga, ga + 4 * WB_GP);
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int ky = k / 3, kx = k % 3;
        // B = X: rows = the tap-shifted positions of pixels (ks, rowh (+4)), columns = n
        const __bf16* xa = xb + ((g.s * ks + ky) * g.hc + g.s * rowh + kx) * WB_XP + colh;
        const bf16x8 b = wb_tr8(xa, xa + 4 * g.s * WB_XP);
        acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[k], 0, 0, 0);
      }
    }
    if (more) wb_put<TX, XV>(g, st, lds + ((atom + 1 - a_lo) & 1) * WB_BUF, tid);
    __syncthreads();
  }
  flush(tile);
}

// K2C: the partials of every tile (32 map channels) summed in workgroup order into dW in the MAP's
// channel order [O][C][9] (the pose weight swap then gives the reference order).  A block owns one
// (tile, o block): it reads each contributor's 9 x 16 x 64 fragment floats in their stored order
// (thread = consecutive floats: coalesced), sums them in registers in workgroup order, parks the sum
// in LDS and writes dW in its own order (9 taps of one (o, n) contiguous) — the direct form read
// the fragments at a 4-KB stride per thread (98 us per call at config 3)
__global__ __launch_bounds__(256) void pwb_reduce_map_k(WbGeom g, const float* __restrict__ partial,
                                                        float* __restrict__ dw) {
  constexpr int NF = 9 * 16 * 64;                   // floats of one wave's fragments
  __shared__ float sm[NF];
  const int t = blockIdx.x;                          // tile: map channels 32 t ..
  const int ob = blockIdx.y;                         // o block (32 o)
  PwGeom pg;                                         // pw_owner's view of the ranges
  pg.natom = g.natom;
  pg.ngroup = g.ngroup;
  const int g0 = pw_owner(pg, (long long)t * g.L), g1 = pw_owner(pg, (long long)(t + 1) * g.L - 1);
  constexpr int PER = NF / 256;                      // 36 floats per thread
  float v[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) v[k] = 0.f;
  for (int grp = g0; grp <= g1; ++grp) {
    const int slot = t - (int)(wb_lo(g, grp) / g.L);
    const float* src = partial + (((size_t)grp * g.slots + slot) * PW_WAVES + ob) * NF + threadIdx.x;
#pragma unroll
    for (int k = 0; k < PER; ++k) v[k] += src[256 * k];
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) sm[threadIdx.x + 256 * k] = v[k];
  __syncthreads();
  for (int e = threadIdx.x; e < 32 * 32 * 9; e += 256) {
    const int tap = e % 9, nl = (e / 9) % 32, ol = e / (9 * 32);
    const int n = 32 * t + nl;
    if (n >= g.C) continue;
    // C/D layout of the 32 x 32 block: row (o) = (r & 3) + 8 (r >> 2) + 4 lh, column (n) = lane & 31
    const int lh = (ol >> 2) & 1, r = (ol & 3) + 4 * (ol >> 3), ln = nl + 32 * lh;
    dw[((size_t)(32 * ob + ol) * g.C + n) * 9 + tap] = sm[(tap * 16 + r) * 64 + ln];
  }
}

// d bias of bf16 G: fixed-order column sums (blocks of PW_BIAS_ROWS rows), then pcw_bias_fin_k
__global__ __launch_bounds__(256) void pwb_bias_k(int rows, const __bf16* __restrict__ gp, float* __restrict__ part) {
  const int r0 = blockIdx.x * PW_BIAS_ROWS;
  const int r1 = r0 + PW_BIAS_ROWS < rows ? r0 + PW_BIAS_ROWS : rows;
  float s = 0.f;
  for (int r = r0; r < r1; r += 8) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = r + k < r1 ? (float)gp[(size_t)(r + k) * PC_O + threadIdx.x] : 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k];
  }
  part[blockIdx.x * PC_O + threadIdx.x] = s;
}

static WbGeom wb_plan(int nimg, int ho, int wo, int hp, int wp, int s, int C) {
  WbGeom g;
  g.nimg = nimg;
  g.ho = ho;
  g.wo = wo;
  g.hp = hp;
  g.wp = wp;
  g.s = s;
  g.C = C;
  g.tc = (wo + WB_TC - 1) / WB_TC;
  g.tiles_img = ((ho + WB_TR - 1) / WB_TR) * g.tc;
  g.L = nimg * g.tiles_img;
  g.ntile = (C + 31) / 32;
  g.natom = g.ntile * g.L;
  const int res = pc_resident();
  g.ngroup = g.natom < res ? g.natom : res;
  const long long range = (g.natom + g.ngroup - 1) / g.ngroup;
  g.slots = (int)((range - 1) / g.L) + 2;
  g.hr = s * (WB_TR - 1) + 3;
  g.hc = s * (WB_TC - 1) + 3;
  return g;
}

// vec: channels per 16-B load of X (bf16 8, fp32 4): C a multiple of it
static bool wb_supported(const WbGeom& g, int vec) {
  if (g.nimg <= 0 || g.ho <= 0 || g.wo <= 0 || (g.s != 1 && g.s != 2) || g.C <= 0 || g.C % vec) return false;
  const long long range = g.natom / g.ngroup;
  return range > 0 && (g.L + range - 1) / range + 1 <= PW_MAXC;   // workgroups meeting one tile (reduce)
}

static PwGeom wb_as_pw(const WbGeom& w, int D) {
  PwGeom g;
  g.nbc = w.nimg;
  g.h = w.ho;
  g.w = w.wo;
  g.ntot = w.C;
  g.D = D;
  g.tc = w.tc;
  g.tiles_img = w.tiles_img;
  g.L = w.L;
  g.ntile = w.ntile;
  g.natom = w.natom;
  g.ngroup = w.ngroup;
  g.slots = w.slots;
  return g;
}

}  // namespace vfd

using namespace vfd;

extern "C" {

size_t vfd_proj_conv_fwd_workspace(const vfd_voxel_desc* d) {
  if (!d || d->D <= 0 || d->h <= 0 || d->w <= 0) return 0;
  return (size_t)pc_plan(*d).ngroup * 2 * PC_FRAG * sizeof(float);
}

int vfd_proj_conv_fwd(const vfd_voxel_desc* d, const float* vox, const float* invK, const float* E,
                      const float* Wq, const float* bias, int out_channels, float* out, float* x_out, void* ws,
                      size_t ws_bytes, void* stream) {
  VFD_REQUIRE(d && vox && invK && E && Wq && bias && out, "proj_conv_fwd: null argument");
  VFD_REQUIRE(d->Cv == PC_CV, "proj_conv_fwd: Cv must be %d (got %d)", PC_CV, d->Cv);
  VFD_REQUIRE(out_channels == PC_O, "proj_conv_fwd: output channels must be %d (got %d)", PC_O, out_channels);
  VFD_REQUIRE(d->B > 0 && d->N > 0 && d->h >= 2 && d->w >= 2 && d->D > 0 && d->D <= 64,
              "proj_conv_fwd: bad shape (h, w >= 2, 0 < D <= 64)");
  VFD_REQUIRE(ws && ws_bytes >= vfd_proj_conv_fwd_workspace(d), "proj_conv_fwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_PROJ_CONV_FWD, s);
  const PcGeom g = pc_plan(*d);
  float* partial = (float*)ws;
  pcv_main_k<<<g.ngroup, PC_THREADS, 0, s>>>(*d, g, vox, invK, E, Wq, partial, x_out);
  pcv_reduce_k<float><<<dim3(g.ntile, PC_FSL), 256, 0, s>>>(*d, g, partial, bias, out);
  return fail_launch("proj_conv_fwd");
}

// bf16 form: same workspace; vox / invK / E fp32, Wq = vfd_weight_fragments mode 3, bias fp32,
// out / x_out bf16 (x_out optional: the frustum features for the weight gradient)
int vfd_proj_conv_fwd_bf16(const vfd_voxel_desc* d, const float* vox, const float* invK, const float* E,
                           const void* Wq, const float* bias, int out_channels, void* out, void* x_out, void* ws,
                           size_t ws_bytes, void* stream) {
  VFD_REQUIRE(d && vox && invK && E && Wq && bias && out, "proj_conv_fwd_bf16: null argument");
  VFD_REQUIRE(d->Cv == PC_CV, "proj_conv_fwd_bf16: Cv must be %d (got %d)", PC_CV, d->Cv);
  VFD_REQUIRE(out_channels == PC_O, "proj_conv_fwd_bf16: output channels must be %d (got %d)", PC_O, out_channels);
  VFD_REQUIRE(d->B > 0 && d->N > 0 && d->h >= 2 && d->w >= 2 && d->D > 0 && d->D <= 64,
              "proj_conv_fwd_bf16: bad shape (h, w >= 2, 0 < D <= 64)");
  VFD_REQUIRE(ws && ws_bytes >= vfd_proj_conv_fwd_workspace(d), "proj_conv_fwd_bf16: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_PROJ_CONV_FWD, s);
  const PcGeom g = pc_plan(*d);
  float* partial = (float*)ws;
  pcvb_main_k<<<g.ngroup, PC_THREADS, 0, s>>>(*d, g, vox, invK, E, (const bf16x8*)Wq, partial, (__bf16*)x_out);
  pcv_reduce_k<__bf16><<<dim3(g.ntile, PC_FSL), 256, 0, s>>>(*d, g, partial, bias, (__bf16*)out);
  return fail_launch("proj_conv_fwd_bf16");
}

#ifndef VFD_PCD_GEN
#define VFD_PCD_GEN 1       // folded fp32 data gradient: 1 = pcdf where its staged rows fit LDS (configs
#endif                      // 2-4: 3.08 vs pcg's 3.15 ms at config 2), pcg otherwise (config 5); 2 = pcg always

// pcg for the folded form: always at VFD_PCD_GEN 2, else where pcdf does not fit
static bool pcd_use_pcg(const vfd_voxel_desc& d) {
  return d.pad_out == 2 && pg_supported<float>(d) && (VFD_PCD_GEN >= 2 || !pf_supported(d));
}

size_t vfd_proj_conv_dgrad_workspace(const vfd_voxel_desc* d) {
  if (!d) return 0;
  if (pcd_use_pcg(*d))
    return (size_t)pg_plan<float>(*d).ngroup * 2 * PG_FRAG * sizeof(float);
  if (d->pad_out == 2) return pf_supported(*d) ? (size_t)pf_plan(*d).ngroup * 2 * PC_FRAG * sizeof(float) : 0;
  if (!pd_supported(*d)) return 0;
  return (size_t)pd_plan(*d).ngroup * 2 * PC_FRAG * sizeof(float);
}

int vfd_proj_conv_dgrad(const vfd_voxel_desc* d, const float* g_pre, const float* Wd, float* dx, void* ws,
                        size_t ws_bytes, void* stream) {
  VFD_REQUIRE(d && g_pre && Wd && dx, "proj_conv_dgrad: null argument");
  const bool gen2 = pcd_use_pcg(*d);
  VFD_REQUIRE(gen2 || (d->pad_out == 2 ? pf_supported(*d) : pd_supported(*d)),
              "proj_conv_dgrad: unsupported shape (Cv = %d, 0 < D <= 64, staged rows in LDS; folded: h >= 6, w >= 64)", PC_CV);
  VFD_REQUIRE(ws && ws_bytes >= vfd_proj_conv_dgrad_workspace(d), "proj_conv_dgrad: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_PROJ_CONV_DGRAD, s);
  if (gen2) {
    const PgGeom g = pg_plan<float>(*d);
    lds_attr(reinterpret_cast<const void*>(pcg_main_k<float, float>), PD_LDS_MAX);
    pcg_main_k<float, float><<<g.ngroup, PC_THREADS, (size_t)2 * g.lds_elems * sizeof(float), s>>>(g, g_pre, Wd, dx,
                                                                                                  (float*)ws);
    pcg_reduce_k<<<dim3(g.ngroup, PC_FSL), 256, 0, s>>>(g, (const float*)ws, dx);
    return fail_launch("proj_conv_dgrad");
  }
  if (d->pad_out == 2) {
    const PfGeom g = pf_plan(*d);
    lds_attr(reinterpret_cast<const void*>(pcdf_main_k), PD_LDS_MAX);
    pcdf_main_k<<<g.ngroup, PC_THREADS, (size_t)2 * g.lds_floats * sizeof(float), s>>>(g, g_pre, Wd, dx, (float*)ws);
    pcdf_reduce_k<<<dim3(g.ngroup, PC_FSL), 256, 0, s>>>(g, (const float*)ws, dx);
    return fail_launch("proj_conv_dgrad");
  }
  const PdGeom g = pd_plan(*d);
  float* partial = (float*)ws;
  const size_t lds = (size_t)2 * g.lds_floats * sizeof(float);
  lds_attr(reinterpret_cast<const void*>(pcd_main_k), PD_LDS_MAX);
  pcd_main_k<<<g.ngroup, PC_THREADS, lds, s>>>(g, g_pre, Wd, dx, partial);
  pcd_reduce_k<<<dim3(g.ngroup, PC_FSL), 256, 0, s>>>(g, partial, dx);
  return fail_launch("proj_conv_dgrad");
}

// bf16 form (config 3): g_pre bf16 [B*N, h, w, O] NHWC, Wd = vfd_weight_fragments_bf16 mode 5, dx fp32
// (the folded interior, pad_out == 2 only)
#ifndef VFD_PCD_BF_2D
#define VFD_PCD_BF_2D 1     // bf16 folded data gradient on 16 x 16 tiles (pch); 0 = pcg's row tiles
#endif

size_t vfd_proj_conv_dgrad_bf16_workspace(const vfd_voxel_desc* d) {
  if (!d || d->pad_out != 2) return 0;
  if (VFD_PCD_BF_2D && ph_supported(*d)) return (size_t)ph_plan(*d).ngroup * 2 * PG_FRAG * sizeof(float);
  if (!pg_supported<__bf16>(*d)) return 0;
  return (size_t)pg_plan<__bf16>(*d).ngroup * 2 * PG_FRAG * sizeof(float);
}

int vfd_proj_conv_dgrad_bf16(const vfd_voxel_desc* d, const void* g_pre, const void* Wd, float* dx, void* ws,
                             size_t ws_bytes, void* stream) {
  VFD_REQUIRE(d && g_pre && Wd && dx, "proj_conv_dgrad_bf16: null argument");
  const bool two_d = VFD_PCD_BF_2D && d->pad_out == 2 && ph_supported(*d);
  VFD_REQUIRE(two_d || (d->pad_out == 2 && pg_supported<__bf16>(*d)),
              "proj_conv_dgrad_bf16: unsupported shape (folded form pad_out = 2, Cv = %d, 0 < D <= 64, staged rows in LDS)",
              PC_CV);
  VFD_REQUIRE(ws && ws_bytes >= vfd_proj_conv_dgrad_bf16_workspace(d), "proj_conv_dgrad_bf16: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_PROJ_CONV_DGRAD, s);
  if (two_d) {
    const PhGeom g = ph_plan(*d);
    pch_main_k<<<g.ngroup, PC_THREADS, 0, s>>>(g, (const __bf16*)g_pre, (const bf16x8*)Wd, dx, (float*)ws);
    pch_reduce_k<<<dim3(g.ngroup, PC_FSL), 256, 0, s>>>(g, (const float*)ws, dx);
    return fail_launch("proj_conv_dgrad_bf16");
  }
  const PgGeom g = pg_plan<__bf16>(*d);
  lds_attr(reinterpret_cast<const void*>(pcg_main_k<__bf16, __bf16>), PD_LDS_MAX);
  pcg_main_k<__bf16, __bf16><<<g.ngroup, PC_THREADS, (size_t)2 * g.lds_elems * sizeof(__bf16), s>>>(
      g, (const __bf16*)g_pre, Wd, dx, (float*)ws);
  pcg_reduce_k<<<dim3(g.ngroup, PC_FSL), 256, 0, s>>>(g, (const float*)ws, dx);
  return fail_launch("proj_conv_dgrad_bf16");
}

size_t vfd_proj_conv_wgrad_workspace(const vfd_voxel_desc* d) {
  if (!d || !pw_supported(*d)) return 0;
  const PwGeom g = pw_plan(*d);
  const int nblk = (g.nbc * g.h * g.w + PW_BIAS_ROWS - 1) / PW_BIAS_ROWS;
  return ((size_t)g.ngroup * g.slots * PW_FRAG + (size_t)nblk * PC_O) * sizeof(float);
}

int vfd_proj_conv_wgrad(const vfd_voxel_desc* d, const float* g_pre, const float* x, float* dw, float* db, void* ws,
                        size_t ws_bytes, void* stream) {
  VFD_REQUIRE(d && g_pre && x && (dw || db), "proj_conv_wgrad: null argument");
  VFD_REQUIRE(pw_supported(*d), "proj_conv_wgrad: unsupported shape (Cv = %d, 0 < D <= 64)", PC_CV);
  VFD_REQUIRE(ws && ws_bytes >= vfd_proj_conv_wgrad_workspace(d), "proj_conv_wgrad: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_PROJ_CONV_WGRAD, s);
  const PwGeom g = pw_plan(*d);
  float* partial = (float*)ws;
  if (dw) {
    pcw_main_k<<<g.ngroup, PC_THREADS, 0, s>>>(g, g_pre, x, partial);
    pcw_reduce_k<<<dim3(PC_O / 4, 2 * ((d->D + PW_DC - 1) / PW_DC)), 256, 0, s>>>(g, partial, dw);
  }
  if (db) {
    float* part = partial + (size_t)g.ngroup * g.slots * PW_FRAG;
    const int rows = g.nbc * g.h * g.w, nblk = (rows + PW_BIAS_ROWS - 1) / PW_BIAS_ROWS;
    pcw_bias_k<<<nblk, PC_O, 0, s>>>(rows, g_pre, part);
    pcw_bias_fin_k<<<PC_O / 4, 256, 0, s>>>(nblk, part, db);
  }
  return fail_launch("proj_conv_wgrad");
}

// bf16 K3C weight / bias gradient (config 3): g_pre bf16 [B*N, h, w, O], x = the bf16 frustum side
// output [B*N, h+2, w+2, D*Cv]; dw [O, Cv*D, 3, 3] fp32 in the reference channel order, db [O] fp32
static WbGeom pwb_k3c(const vfd_voxel_desc& d) {
  return wb_plan(d.B * d.N, d.h, d.w, d.h + 2, d.w + 2, 1, d.D * PC_CV);
}

size_t vfd_proj_conv_wgrad_bf16_workspace(const vfd_voxel_desc* d) {
  if (!d || d->Cv != PC_CV || d->D <= 0 || d->D > 64 || d->B <= 0 || d->N <= 0 || d->h < 1 || d->w < 1) return 0;
  const WbGeom g = pwb_k3c(*d);
  if (!wb_supported(g, 8)) return 0;
  const int nblk = (g.nimg * g.ho * g.wo + PW_BIAS_ROWS - 1) / PW_BIAS_ROWS;
  return ((size_t)g.ngroup * g.slots * PW_FRAG + (size_t)nblk * PC_O) * sizeof(float);
}

int vfd_proj_conv_wgrad_bf16(const vfd_voxel_desc* d, const void* g_pre, const void* x, float* dw, float* db,
                             void* ws, size_t ws_bytes, void* stream) {
  VFD_REQUIRE(d && g_pre && x && (dw || db), "proj_conv_wgrad_bf16: null argument");
  const size_t need = vfd_proj_conv_wgrad_bf16_workspace(d);
  VFD_REQUIRE(need, "proj_conv_wgrad_bf16: unsupported shape (Cv = %d, 0 < D <= 64)", PC_CV);
  VFD_REQUIRE(ws && ws_bytes >= need, "proj_conv_wgrad_bf16: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_PROJ_CONV_WGRAD, s);
  const WbGeom g = pwb_k3c(*d);
  float* partial = (float*)ws;
  if (dw) {
    pwb_main_k<__bf16><<<g.ngroup, PC_THREADS, 0, s>>>(g, (const __bf16*)g_pre, (const __bf16*)x, partial);
    const PwGeom pg = wb_as_pw(g, d->D);
    pcw_reduce_k<<<dim3(PC_O / 4, 2 * ((d->D + PW_DC - 1) / PW_DC)), 256, 0, s>>>(pg, partial, dw);
  }
  if (db) {
    float* part = partial + (size_t)g.ngroup * g.slots * PW_FRAG;
    const int rows = g.nimg * g.ho * g.wo, nblk = (rows + PW_BIAS_ROWS - 1) / PW_BIAS_ROWS;
    pwb_bias_k<<<nblk, PC_O, 0, s>>>(rows, (const __bf16*)g_pre, part);
    pcw_bias_fin_k<<<PC_O / 4, 256, 0, s>>>(nblk, part, db);
  }
  return fail_launch("proj_conv_wgrad_bf16");
}

// bf16 K2C weight / bias gradient (config 3; the pose reduce_dim[0], stride d->stride): g_pre bf16
// [B, Ho, Wo, 256], x = the fp32 reflect-padded BEV map [B, H, W, C] (rounded to bf16 as staged);
// dw_map [256, C, 3, 3] fp32 in the MAP's channel order (the caller swaps it to the reference order),
// db [256] fp32
size_t vfd_pad_conv_wgrad_bf16_workspace(const vfd_conv_desc* d) {
  if (!d || d->out_channels != PC_O || d->B <= 0 || d->H < 3 || d->W < 3 || (d->stride != 1 && d->stride != 2)) return 0;
  const int ho = (d->H - 3) / d->stride + 1, wo = (d->W - 3) / d->stride + 1;
  const WbGeom g = wb_plan(d->B, ho, wo, d->H, d->W, d->stride, d->C);
  if (!wb_supported(g, 4)) return 0;
  const int nblk = (g.nimg * g.ho * g.wo + PW_BIAS_ROWS - 1) / PW_BIAS_ROWS;
  return ((size_t)g.ngroup * g.slots * PW_FRAG + (size_t)nblk * PC_O) * sizeof(float);
}

int vfd_pad_conv_wgrad_bf16_t(const vfd_conv_desc* d, const void* g_pre, const void* x, int dtype_x, float* dw_map,
                              float* db, void* ws, size_t ws_bytes, void* stream) {
  VFD_REQUIRE(d && g_pre && x && (dw_map || db), "pad_conv_wgrad_bf16: null argument");
  VFD_REQUIRE(dtype_x == 0 || dtype_x == 1, "pad_conv_wgrad_bf16: dtype_x %d (0 fp32, 1 bf16)", dtype_x);
  const size_t need = vfd_pad_conv_wgrad_bf16_workspace(d);
  VFD_REQUIRE(need, "pad_conv_wgrad_bf16: unsupported shape (C %% 4 == 0, stride 1 or 2, %d outputs)", PC_O);
  VFD_REQUIRE(ws && ws_bytes >= need, "pad_conv_wgrad_bf16: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_PAD_CONV_WGRAD, s);
  const int ho = (d->H - 3) / d->stride + 1, wo = (d->W - 3) / d->stride + 1;
  const WbGeom g = wb_plan(d->B, ho, wo, d->H, d->W, d->stride, d->C);
  float* partial = (float*)ws;
  if (dw_map) {
    if (dtype_x == 0)
      pwb_main_k<float><<<g.ngroup, PC_THREADS, 0, s>>>(g, (const __bf16*)g_pre, (const float*)x, partial);
    else if (d->C % 8 == 0)
      pwb_main_k<__bf16, 8><<<g.ngroup, PC_THREADS, 0, s>>>(g, (const __bf16*)g_pre, (const __bf16*)x, partial);
    else
      pwb_main_k<__bf16, 4><<<g.ngroup, PC_THREADS, 0, s>>>(g, (const __bf16*)g_pre, (const __bf16*)x, partial);
    pwb_reduce_map_k<<<dim3(g.ntile, PC_O / 32), 256, 0, s>>>(g, partial, dw_map);
  }
  if (db) {
    float* part = partial + (size_t)g.ngroup * g.slots * PW_FRAG;
    const int rows = g.nimg * g.ho * g.wo, nblk = (rows + PW_BIAS_ROWS - 1) / PW_BIAS_ROWS;
    pwb_bias_k<<<nblk, PC_O, 0, s>>>(rows, (const __bf16*)g_pre, part);
    pcw_bias_fin_k<<<PC_O / 4, 256, 0, s>>>(nblk, part, db);
  }
  return fail_launch("pad_conv_wgrad_bf16");
}

int vfd_pad_conv_wgrad_bf16(const vfd_conv_desc* d, const void* g_pre, const float* x, float* dw_map, float* db,
                            void* ws, size_t ws_bytes, void* stream) {
  return vfd_pad_conv_wgrad_bf16_t(d, g_pre, x, 0, dw_map, db, ws, ws_bytes, stream);
}

}  // extern "C"
