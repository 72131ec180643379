// K2C — reduce_dim's first conv of the POSE fusion (network/volumetric_fusionnet.py:59-60,
// 338-343): a 3x3, stride-s convolution of the reflect-padded channels-last BEV map K2 writes
// ([B, Hp, Wp, Cin], Cin = (C+1)*Z = 5140 at config 2) into O = 256 channels, + bias,
// LeakyReLU(0.1), stored as the reflect-padded NHWC input of reduce_dim's second conv.
//
//   Y[b, y, x, o] = lrelu(bias[o] + sum_{ty, tx, c} W[o, c, ty, tx] * Xp[b, s*y + ty, s*x + tx, c])
//
// fp32 MFMA implicit GEMM (v_mfma_f32_32x32x2_f32): M = output pixels (row-major, 128 per tile),
// N = O = 256 (4 compute waves x 64), K = 9 * Cin.  The GEMM is short and deep (M = 2500 at
// config 2: 20 tiles for 256 CUs), so the K dimension is split stream-K style: an atom = (tile,
// 16-channel chunk); loader waves stage the chunk's input rows under the tile (hrows x Wp
// positions) into one half of a double-buffered LDS image while the compute waves run the
// previous atom's 9 taps x 4 channel quads.  Split tiles are summed by `ppc_reduce_k` in
// workgroup order (deterministic), which also applies the epilogue to every tile.
#include <type_traits>

#include "vfd_common.h"

namespace vfd {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int PP_O = 256;                       // output channels (4 waves x 64)
constexpr int PP_WAVES = 4;
constexpr int PP_THREADS = 512;                 // 4 compute + 4 loader waves
constexpr int PP_PIX = 128;                     // output pixels per tile
constexpr int PP_CC = 16;                       // input channels per atom
constexpr int PP_XS = PP_CC + 4;                // LDS floats per staged position (16-B rows)
constexpr int PP_ITERS = 9 * (PP_CC / 4);       // (tap, quad) iterations per atom
constexpr int PP_PF = 4;                        // weight-fragment prefetch distance
constexpr int PP_FRAG = PP_PIX * PP_O;          // floats of one tile's partial
constexpr int PP_LDS_MAX = 160 * 1024;
constexpr int PP_MAXC = 96;                     // contributors of one tile
constexpr int PP_FSL = 32;                      // fragment slices per tile in the reduce
#ifndef VFD_PP_ALIGN
#define VFD_PP_ALIGN 1                          // tile-aligned stream-K splits + XCD numbering (pp_plan)
#endif

// workgroup -> stream-K group: with ngroup % 8 == 0 XCD k (workgroups k, k + 8, ...) takes the
// contiguous groups [k ngroup / 8, (k+1) ngroup / 8)
struct PpGeom {
  int B, hp, wp, cin, s, ho, wo, mimg, mtiles, nchunk, cq, ntile, natom, ngroup, hrows, lds_floats, xcd;
};

__device__ __forceinline__ int pp_group(const PpGeom& g) {
  return g.xcd ? (blockIdx.x % 8) * (g.ngroup / 8) + blockIdx.x / 8 : blockIdx.x;
}

__host__ __device__ inline int pp_lo(const PpGeom& g, int grp) {
  return (int)(((long long)grp * g.natom) / g.ngroup);
}

struct PpTile {
  int b, m0, ymin;
};

__device__ __forceinline__ PpTile pp_tile(const PpGeom& g, int t) {
  PpTile r;
  r.b = t / g.mtiles;
  r.m0 = (t - r.b * g.mtiles) * PP_PIX;
  r.ymin = r.m0 / g.wo;
  return r;
}

// loader waves (tid 0..255): input rows s*ymin .. s*ymin + hrows - 1 (all Wp columns), channels
// ch*CC .. ch*CC + CC - 1 (zero past Cin)
template <int CC>
__device__ __forceinline__ void pp_stage(const PpGeom& g, float* __restrict__ dst, const float* __restrict__ x,
                                         int atom, int tid) {
  constexpr int QP = CC / 4, PPP = 256 / QP, XS = CC + 4;
  const int t = atom / g.nchunk, ch = atom - t * g.nchunk;
  const PpTile tl = pp_tile(g, t);
  const int npos = g.hrows * g.wp;
  const int q = tid % QP;
  const int c = ch * CC + 4 * q;
  const int r0 = g.s * tl.ymin;
  const float* src = x + ((size_t)tl.b * g.hp + r0) * g.wp * g.cin + c;
  const bool cok = c < g.cin;
  // positions p < plim lie in rows r0 + p / wp < hp (no per-position division)
  const int plim = min(npos, (g.hp - r0) * g.wp);
  for (int p0 = tid / QP; p0 < npos; p0 += 4 * PPP) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = p0 + PPP * u;
      v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (cok && p < plim)
        v[u] = *reinterpret_cast<const float4*>(src + (unsigned)(p * g.cin));   // p * cin < 2^31
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = p0 + PPP * u;
      if (p < npos) *reinterpret_cast<float4*>(dst + p * XS + 4 * q) = v[u];
    }
  }
}

// bias + LeakyReLU(0.1) of output pixel m (of image b), stored at every reflect-pad copy
template <typename TO>
__device__ __forceinline__ void pp_store(const PpGeom& g, TO* __restrict__ out, const float* __restrict__ bias,
                                         int b, int m, int o, float acc) {
  if (m >= g.mimg) return;
  const int y = m / g.wo, xx = m - y * g.wo;
  float v = acc + bias[o];
  v = v > 0.f ? v : v * 0.1f;
  int rows[3], cols[3], nr, nc;
  pad_sets(y, g.ho, true, rows, &nr);
  pad_sets(xx, g.wo, true, cols, &nc);
  TO* ob = out + (size_t)b * (g.ho + 2) * (g.wo + 2) * PP_O + o;
  for (int i = 0; i < nr; ++i)
    for (int j = 0; j < nc; ++j) ob[((size_t)rows[i] * (g.wo + 2) + cols[j]) * PP_O] = (TO)v;
}

// Weight layout Wf: [9 taps][cq = Cin_pad/4 quads][O][2 (h)][2 (s)], c = 4*quad + 2*h + s
// (channels past Cin zero).  CC = channels per atom: 16, or 8 where the staged rows of 16 do not
// fit LDS (config 5's 202-wide BEV map).
template <int CC>
__global__ __launch_bounds__(PP_THREADS, 2) void ppc_main_k(PpGeom g, const float* __restrict__ x,
                                                           const float* __restrict__ Wf,
                                                           const float* __restrict__ bias,
                                                           float* __restrict__ out,
                                                           float* __restrict__ partial) {
  constexpr int XS = CC + 4, ITERS = 9 * (CC / 4), PF = CC / 4 < PP_PF ? CC / 4 : PP_PF;
  extern __shared__ float pp_lds[];
  const int grp = pp_group(g);
  const int a_lo = pp_lo(g, grp), a_hi = pp_lo(g, grp + 1);
  if (a_lo >= a_hi) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool compute = wv < PP_WAVES;
  if (!compute) pp_stage<CC>(g, pp_lds, x, a_lo, threadIdx.x - 64 * PP_WAVES);
  __syncthreads();
  if (!compute) {
    for (int atom = a_lo; atom < a_hi; ++atom) {
      if (atom + 1 < a_hi)
        pp_stage<CC>(g, pp_lds + ((atom + 1 - a_lo) & 1) * g.lds_floats, x, atom + 1, threadIdx.x - 64 * PP_WAVES);
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
  const float2* wlane = reinterpret_cast<const float2*>(Wf) + (size_t)(wv * 64 + li) * 2 + lh;
  float2 bq[PF][2];
  int pf_atom = a_lo, pf_it = 0;
  int pf_ch = a_lo % g.nchunk;                        // the prefetched atom's channel chunk
  auto prefetch = [&](int slot) {
    if (pf_atom < a_hi) {
      const int tap = pf_it / (CC / 4), q = pf_it % (CC / 4);
      const float2* w = wlane + (size_t)(tap * g.cq + pf_ch * (CC / 4) + q) * (2 * PP_O);
      bq[slot][0] = w[0];
      bq[slot][1] = w[64];
      if (++pf_it == ITERS) {
        pf_it = 0;
        ++pf_atom;
        pf_ch = pf_ch + 1 == g.nchunk ? 0 : pf_ch + 1;
      }
    }
  };
#pragma unroll
  for (int k = 0; k < PF; ++k) prefetch(k);
  int cur_t = -1;
  int aoff[4];                                        // the lane's pixels' LDS offsets (per tile)
  for (int atom = a_lo; atom < a_hi; ++atom) {
    const int t = atom / g.nchunk, ch = atom - t * g.nchunk;
    const PpTile tl = pp_tile(g, t);
    if (t != cur_t) {                                 // pixel geometry once per tile
      cur_t = t;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        int m = tl.m0 + 32 * a + li;
        m = m < g.mimg ? m : g.mimg - 1;               // pixels past the image: computed, never stored
        const int y = m / g.wo, xx = m - y * g.wo;
        aoff[a] = (g.s * (y - tl.ymin) * g.wp + g.s * xx) * XS + 2 * lh;
      }
    }
    const float* xb = pp_lds + ((atom - a_lo) & 1) * g.lds_floats;
    float2 afc[4], afn[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) afc[a] = *reinterpret_cast<const float2*>(&xb[aoff[a]]);
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap - 3 * ky;
      const float* xt = xb + (ky * g.wp + kx) * XS;
      const int tn = tap + 1, kyn = tn / 3, kxn = tn - 3 * kyn;
      const float* xn = xb + (kyn * g.wp + kxn) * XS;
#pragma unroll
      for (int q = 0; q < CC / 4; ++q) {
        const int ring = q % PF;                      // (CC / 4) % PF == 0: static ring slots
        const float2 b0 = bq[ring][0], b1 = bq[ring][1];
        prefetch(ring);
        if (q < CC / 4 - 1) {
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
    if (ch == g.nchunk - 1 || atom == a_hi - 1) {
      // a tile whole inside this range goes to its own buffer, a split one to partial slot 0 (the
      // range's first tile) or 1 (its last)
      const int ts = t * g.nchunk;
      const size_t buf = (ts >= a_lo && ts + g.nchunk <= a_hi) ? (size_t)g.ngroup * 2 + t
                                                              : (size_t)grp * 2 + (t == a_lo / g.nchunk ? 0 : 1);
      float* dst = partial + buf * PP_FRAG + (size_t)wv * (PP_FRAG / PP_WAVES);
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

// ---------------------------------------------------------------------------------------------
// bf16 form (config 3): the same tiles / stream-K ranges, 32-channel atoms staged as bf16 (the
// fp32 map rounded to nearest even by the loader waves), v_mfma_f32_32x32x16_bf16 with fp32
// accumulation: an atom is 9 taps x 2 sixteen-channel steps of 8 MFMAs per compute wave; lane
// (r, h) of a pixel block reads channels 16q + 8h .. +7 of its input position (one 16-B LDS read).
// Weights: vfd_weight_fragments_bf16 mode 4, [9][cpad/16][O/32][64 lanes][8], lane (r, h) of
// block ob holding W[32 ob + r][16 q + 8 h + j] (cpad = C rounded up to 32, zero past C).
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int PPB_CC = 32;                      // input channels per atom (16 where 32 do not fit LDS)
constexpr int PPB_XS = PPB_CC + 8;              // bf16 per staged position (80 B: 16-B aligned)
#ifndef VFD_PPB_PF
#define VFD_PPB_PF 3                            // weight-fragment prefetch distance (steps; divides 18)
#endif
#ifndef VFD_PPB_U
#define VFD_PPB_U 16                            // loader: 16-B loads in flight per lane
#endif
// The staged rows (~120 KB of the fp32 map per atom) and the weight steps (147 KB) both come from
// L2 / HBM at ~2 us latency: a CU keeps U x 4 KB of rows and PF steps of fragments in flight, the
// loader waves having the VGPRs the compute waves need anyway (one workgroup per CU).

// one channel quad of the map as bf16: the fp32 map rounded to nearest even (16-B loads), or the
// bf16 map K2 writes under config 3 (8-B loads of the same rounded values: C % 4 == 0 keeps a quad
// 8-B aligned at any position)
template <typename TX>
struct PbQuad;
template <>
struct PbQuad<float> {
  typedef float4 V;
  static __device__ __forceinline__ V zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
  static __device__ __forceinline__ V load(const float* p) { return *reinterpret_cast<const float4*>(p); }
  static __device__ __forceinline__ bf16x4 cvt(const V& v) {
    bf16x4 b;
    b[0] = (__bf16)v.x;
    b[1] = (__bf16)v.y;
    b[2] = (__bf16)v.z;
    b[3] = (__bf16)v.w;
    return b;
  }
};
template <>
struct PbQuad<__bf16> {
  typedef bf16x4 V;
  static __device__ __forceinline__ V zero() {
    V z;
#pragma unroll
    for (int e = 0; e < 4; ++e) z[e] = (__bf16)0.f;
    return z;
  }
  static __device__ __forceinline__ V load(const __bf16* p) { return *reinterpret_cast<const bf16x4*>(p); }
  static __device__ __forceinline__ bf16x4 cvt(const V& v) { return v; }
};

template <int CC, typename TX>
__device__ __forceinline__ void ppb_stage(const PpGeom& g, __bf16* __restrict__ dst, const TX* __restrict__ x,
                                          int atom, int tid) {
  typedef PbQuad<TX> PQ;
  // loads in flight per lane: U 16-B vectors of the fp32 map, 2U 8-B vectors of the bf16 one
  constexpr int QP = CC / 4, PPP = 256 / QP, XS = CC + 8, U = VFD_PPB_U * 4 / (int)sizeof(TX);
  const int nchunk = (g.cin + CC - 1) / CC;
  const int t = atom / nchunk, ch = atom - t * nchunk;
  const PpTile tl = pp_tile(g, t);
  const int npos = g.hrows * g.wp;
  const int q = tid % QP;                       // channel quad of the chunk
  const int c = ch * CC + 4 * q;
  const int r0 = g.s * tl.ymin;
  const TX* src = x + ((size_t)tl.b * g.hp + r0) * g.wp * g.cin + c;
  const bool cok = c < g.cin;                   // cin % 4 == 0: a quad is all in or all out
  const int pval = min(npos, (g.hp - r0) * g.wp);  // positions inside the map
  for (int p0 = tid / QP; p0 < npos; p0 += U * PPP) {
    typename PQ::V v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + PPP * u;
      v[u] = PQ::zero();
      if (cok && p < pval) v[u] = PQ::load(src + (unsigned)(p * g.cin));   // p * cin < 2^31: 32-bit offsets
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + PPP * u;
      if (p < npos) *reinterpret_cast<bf16x4*>(dst + p * XS + 4 * q) = PQ::cvt(v[u]);
    }
  }
}

template <int CC, typename TX>
__global__ __launch_bounds__(PP_THREADS, 2) void ppcb_main_k(PpGeom g, const TX* __restrict__ x,
                                                            const bf16x8* __restrict__ Wf,
                                                            float* __restrict__ partial) {
  constexpr int XS = CC + 8, SPT = CC / 16, STEPS = 9 * SPT, PF = SPT == 2 ? VFD_PPB_PF : 3;
  static_assert(STEPS % PF == 0, "prefetch ring");
  extern __shared__ __attribute__((aligned(16))) __bf16 ppb_lds[];
  const int grp = pp_group(g);
  const int a_lo = pp_lo(g, grp), a_hi = pp_lo(g, grp + 1);
  if (a_lo >= a_hi) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool compute = wv < PP_WAVES;
  const int lds_elems = g.hrows * g.wp * XS;
  if (!compute) ppb_stage<CC, TX>(g, ppb_lds, x, a_lo, threadIdx.x - 64 * PP_WAVES);
  __syncthreads();
  if (!compute) {
    for (int atom = a_lo; atom < a_hi; ++atom) {
      if (atom + 1 < a_hi)
        ppb_stage<CC, TX>(g, ppb_lds + ((atom + 1 - a_lo) & 1) * lds_elems, x, atom + 1, threadIdx.x - 64 * PP_WAVES);
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
  const int nchunk = g.nchunk;                  // CC-channel chunks (host-set for the bf16 form)
  const int nq16 = (g.cin + 31) / 32 * 2;       // 16-channel steps per tap of the fragment copy (C to 32)
  // weight fragments addressed as the uniform base + a 32-bit per-lane byte offset (the fragment
  // copy is < 4 GB): one VGPR per in-flight step instead of a 64-bit pointer
  const char* wbase = reinterpret_cast<const char*>(Wf);
  constexpr unsigned QS = (PP_O / 32) * 64 * 16;   // bytes of one 16-channel step of the copy
  const unsigned tstride = (unsigned)nq16 * QS;     // one tap
  const unsigned wlane = (unsigned)(2 * wv * 64 + lane) * 16u;
  auto wsrc = [&](int atom) { return wlane + (unsigned)(atom % nchunk) * SPT * QS; };
  // B fragments of step s (tap s / SPT, step s % SPT) of the atom whose fragments start at w
  auto wld = [&](unsigned w, int s, bf16x8* b) {
    const unsigned o = w + (unsigned)(s / SPT) * tstride + (unsigned)(s % SPT) * QS;
    b[0] = *reinterpret_cast<const bf16x8*>(wbase + o);
    b[1] = *reinterpret_cast<const bf16x8*>(wbase + o + 64u * 16u);
  };
  bf16x8 bq[PF][2];
  unsigned wc = wsrc(a_lo);
#pragma unroll
  for (int k = 0; k < PF; ++k) wld(wc, k, bq[k]);
  int cur_t = -1;
  int aoff[4];                                        // the lane's pixels' LDS offsets (per tile)
  for (int atom = a_lo; atom < a_hi; ++atom) {
    const bool more = atom + 1 < a_hi;
    const unsigned wn = more ? wsrc(atom + 1) : 0u;
    const int t = atom / nchunk, ch = atom - t * nchunk;
    const PpTile tl = pp_tile(g, t);
    if (t != cur_t) {                                 // pixel geometry once per tile
      cur_t = t;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        int m = tl.m0 + 32 * a + li;
        m = m < g.mimg ? m : g.mimg - 1;               // pixels past the image: computed, never stored
        const int y = m / g.wo, xx = m - y * g.wo;
        aoff[a] = (g.s * (y - tl.ymin) * g.wp + g.s * xx) * XS + 8 * lh;
      }
    }
    const __bf16* xb = ppb_lds + ((atom - a_lo) & 1) * lds_elems;
#pragma unroll 1
    for (int s0 = 0; s0 < STEPS; s0 += PF)
#pragma unroll
    for (int ring = 0; ring < PF; ++ring) {         // STEPS % PF == 0: static ring slots across atoms
      const int st = s0 + ring;
      const int tap = st / SPT, q = st % SPT, ky = tap / 3, kx = tap - 3 * ky;
      const __bf16* xt = xb + (ky * g.wp + kx) * XS;
      bf16x8 af[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) af[a] = *reinterpret_cast<const bf16x8*>(&xt[aoff[a] + 16 * q]);
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        acc[a][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bq[ring][0], acc[a][0], 0, 0, 0);
        acc[a][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bq[ring][1], acc[a][1], 0, 0, 0);
      }
      // the refill lands in the slot the MFMAs above just read (no register copy of the slot)
      if (st + PF < STEPS)
        wld(wc, st + PF, bq[ring]);
      else if (more)
        wld(wn, st + PF - STEPS, bq[ring]);
      // keep the scheduler from hoisting later steps' LDS reads above these MFMAs (register
      // pressure: the prefetch ring, not the A fragments, is what should hold VGPRs)
      __builtin_amdgcn_sched_barrier(0);
    }
    wc = wn;
    __syncthreads();                                  // buffer handed back to the loader waves
    if (ch == nchunk - 1 || atom == a_hi - 1) {
      const int ts = t * nchunk;
      const size_t buf = (ts >= a_lo && ts + nchunk <= a_hi) ? (size_t)g.ngroup * 2 + t
                                                            : (size_t)grp * 2 + (t == a_lo / nchunk ? 0 : 1);
      float* dst = partial + buf * PP_FRAG + (size_t)wv * (PP_FRAG / PP_WAVES);
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

// every tile: its own buffer (finished inside one workgroup) or the partials of every workgroup
// meeting it, summed in workgroup order; + bias, LeakyReLU, reflect-padded store
template <typename TO>
__global__ __launch_bounds__(256) void ppc_reduce_k(PpGeom g, const float* __restrict__ partial,
                                                    const float* __restrict__ bias, TO* __restrict__ out) {
  __shared__ int contrib[PP_MAXC];
  __shared__ int ncontrib;
  const int t = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int a0 = t * g.nchunk, a1 = a0 + g.nchunk;
  if (threadIdx.x == 0) {
    int gg = (int)(((long long)a0 * g.ngroup) / g.natom);
    while (gg > 0 && pp_lo(g, gg) > a0) --gg;
    while (pp_lo(g, gg + 1) <= a0) ++gg;
    int n = 0;
    if (pp_lo(g, gg + 1) >= a1) {                     // whole inside group gg: the tile's own buffer
      contrib[n++] = g.ngroup * 2 + t;
    } else {                                          // split tile
      for (; gg < g.ngroup && n < PP_MAXC; ++gg) {
        const int lo = pp_lo(g, gg), hi = pp_lo(g, gg + 1);
        if (lo >= a1) break;
        if (hi <= a0 || lo >= hi) continue;
        contrib[n++] = gg * 2 + (t == lo / g.nchunk ? 0 : 1);
      }
    }
    ncontrib = n;
  }
  __syncthreads();
  const int nc = ncontrib;
  const PpTile tl = pp_tile(g, t);
  constexpr int FPS = 4 * 2 * 16 / PP_FSL;
  float su[FPS];
  frag_sums<FPS>(partial, contrib, nc, PP_FRAG, (size_t)wv * (PP_FRAG / PP_WAVES) + (blockIdx.y * FPS * 64 + lane), su);
#pragma unroll
  for (int u = 0; u < FPS; ++u) {
    const int f = blockIdx.y * FPS + u;
    const int a = f >> 5, bb = (f >> 4) & 1, r = f & 15;
    const int m = tl.m0 + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    pp_store(g, out, bias, tl.b, m, wv * 64 + bb * 32 + (lane & 31), su[u]);
  }
}

static int pp_resident() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  return cus;
}

// align: tile-aligned splits + XCD numbering (the bf16 forward: 441 vs 476 us at config 3; the fp32
// forward is MFMA-bound and a little faster without, 550 vs 557 us at config 2)
static bool pp_plan(const vfd_conv_desc& d, PpGeom* out, int cc = PP_CC, int xs_bytes = PP_XS * 4, bool align = false) {
  if (d.B <= 0 || d.C <= 0 || d.C % 4 || d.stride < 1 || d.stride > 2 || d.H < 3 || d.W < 3 ||
      d.out_channels != PP_O)
    return false;
  PpGeom g;
  g.B = d.B;
  g.hp = d.H;
  g.wp = d.W;
  g.cin = d.C;
  g.s = d.stride;
  g.ho = (d.H - 3) / d.stride + 1;
  g.wo = (d.W - 3) / d.stride + 1;
  if (g.ho < 2 || g.wo < 2) return false;
  g.mimg = g.ho * g.wo;
  g.mtiles = (g.mimg + PP_PIX - 1) / PP_PIX;
  g.nchunk = (d.C + cc - 1) / cc;
  g.cq = (d.C + 15) / 16 * 4;            // channel quads per tap of the fp32 fragment copy (C rounded to 16)
  g.ntile = g.B * g.mtiles;
  g.natom = g.ntile * g.nchunk;
  // output rows under 128 consecutive pixels, and the input rows they read
  const int orows = 1 + (g.wo - 1 + PP_PIX - 1) / g.wo;
  g.hrows = g.s * (orows - 1) + 3;
  g.lds_floats = g.hrows * g.wp * (xs_bytes / 4);
  if ((size_t)2 * g.hrows * g.wp * xs_bytes > PP_LDS_MAX) return false;
  if ((size_t)g.hrows * g.wp * g.cin >= ((size_t)1 << 31)) return false;   // loaders' 32-bit offsets
  // ranges of >= ceil(nchunk / (PP_MAXC - 2)) atoms keep a tile's contributors <= PP_MAXC - 1
  const int res = pp_resident();
  const int min_range = (g.nchunk + PP_MAXC - 3) / (PP_MAXC - 2);
  int most = g.natom / min_range;
  most = most > 0 ? most : 1;
  g.ngroup = res < most ? res : most;
  g.xcd = 0;
#if VFD_PP_ALIGN
  // fewer tiles than CUs: every tile cut into the same ksplit chunk ranges (group t * ksplit + j
  // takes chunks [j nchunk / ksplit, (j+1) nchunk / ksplit) of tile t), so the groups of one split
  // read the same weight fragments at the same time; with the XCD numbering of the main kernels
  // the tiles of one XCD share its L2 copy instead of every CU streaming its own from HBM / MALL
  if (align && g.ntile <= res) {
    int ks = res / g.ntile;
    ks = ks < g.nchunk ? ks : g.nchunk;
    ks = ks < PP_MAXC - 1 ? ks : PP_MAXC - 1;
    g.ngroup = g.ntile * ks;
  }
  g.xcd = align && g.ngroup % 8 == 0;
#endif
  *out = g;
  return true;
}

// 16-byte vectors of G (fp32 4 channels, bf16 8), widened to fp32; put<T> rounds once to the LDS type
template <typename TG>
struct PgVecP;
template <>
struct PgVecP<float> {
  static constexpr int CH = 4;
  typedef float4 V;
  static __device__ __forceinline__ V zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
  static __device__ __forceinline__ V load(const float* p) { return *reinterpret_cast<const float4*>(p); }
  template <typename T>
  static __device__ __forceinline__ void put(T* dst, const V& v) { st4(dst, v); }
};
template <>
struct PgVecP<__bf16> {
  static constexpr int CH = 8;
  typedef bf16x8 V;
  static __device__ __forceinline__ V zero() {
    V z;
#pragma unroll
    for (int e = 0; e < 8; ++e) z[e] = (__bf16)0.f;
    return z;
  }
  static __device__ __forceinline__ V load(const __bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
  template <typename T>
  static __device__ __forceinline__ void put(T* dst, const V& v) {
    static_assert(sizeof(T) == 2, "bf16 G staged as bf16");
    *reinterpret_cast<bf16x8*>(dst) = v;
  }
};

// =============================================================================================
// K2C data gradient ("ppd"): d of the stride-s 3x3 conv w.r.t. its reflect-padded input map, the
// backward of ppc_main_k (volumetric_fusionnet.py:59-60, 338-343; the reference's cudnn backward-data
// of reduce_dim[0] under DDP):
//
//   dXp[b, Y, X, c] = sum_{ky, kx: Y = s y + ky, X = s x + kx} sum_o G[b, y, x, o] W[o, c, ky, kx]
//
// For stride 2 a padded position's taps depend on its parity class (Y % 2, X % 2): even rows take
// ky in {0, 2} (G rows Y/2 and Y/2 - 1), odd rows ky = 1 (G row (Y-1)/2); columns alike — 4, 2, 2
// and 1 taps.  Positions are tiled by class: a tile = 256 consecutive positions of one class grid
// (class row i -> Y = 2i + py) of one image, so every pixel of a tile has the same tap list; M =
// those positions, N = 128 map channels per tile (4 waves x 32), K = taps x O.  Atom = (tile,
// OC-channel chunk of O), its trip count = taps x OC / (MFMA k); stream-K ranges are cut in WORK
// units (an atom of a t-tap class costs t) so every workgroup gets the same MFMA count.  The loader
// waves stage the G rows under the tile (rows i0 - 1 .. i1, columns -1 .. wo - 1, zero outside) for
// the atom's chunk; compute waves as pcg (projconv.hip): 8 pixel blocks x one 32-channel block,
// B fragments from the weight's data-gradient copy (vfd_weight_fragments mode 2 with Cv = C1,
// D = Z over the map's channel order; bf16: mode 5 of it), PF steps ahead.  Stride 1 is the same
// with one class of 9 taps.  Whole tiles are stored directly (every padded position belongs to
// exactly one class, so dXp is written in full, zeros included); split tiles summed in group order
// by ppd_reduce_k (deterministic).
#ifndef VFD_PD_U
#define VFD_PD_U 12                             // loader: 16-B loads in flight per lane (one batch per atom)
#endif
#ifndef VFD_PD_BF_PF
#define VFD_PD_BF_PF 4                          // bf16 B-fragment prefetch distance (steps: one tap ahead)
#endif
template <typename T>
struct PdCfg;
template <>
struct PdCfg<float> {
  static constexpr int OC = 16, XS = 20, STEPS = 4, PF = 4;   // o per atom, LDS elems / position, k-steps per tap,
};                                                            // B prefetch distance (steps, <= STEPS)
template <>
struct PdCfg<__bf16> {
  static constexpr int OC = 64, XS = 72, STEPS = 4, PF = VFD_PD_BF_PF;
};

constexpr int PD2_PIX = 256;                    // positions per tile (8 blocks of 32)
constexpr int PD2_N = 128;                      // map channels per tile (4 waves x 32)
constexpr int PD2_FRAG = PD2_PIX * PD2_N;

struct PdcGeom {
  int B, hp, wp, cin, ho, wo, s, np, ntn, och;
  int nclass, py[4], px[4], hc[4], wc[4], tpc[4], ntap[4], ct_start[5], cu_start[5];
  int tiles_nt, units_nt, ntile, natom, ngroup, hrows, cols, lds_elems;
  long long units;
};

__host__ __device__ inline int pdc_class(const PdcGeom& g, int tl) {
  int c = 0;
  while (c + 1 < g.nclass && tl >= g.ct_start[c + 1]) ++c;
  return c;
}

// first atom whose work-unit start is >= u
__host__ __device__ inline int pdc_atom_at(const PdcGeom& g, long long u) {
  if (u >= g.units) return g.natom;
  const int nt = (int)(u / g.units_nt);
  const int ru = (int)(u - (long long)nt * g.units_nt);
  int c = 0;
  while (c + 1 < g.nclass && ru >= g.cu_start[c + 1]) ++c;
  const int k = (ru - g.cu_start[c] + g.ntap[c] - 1) / g.ntap[c];
  return (nt * g.tiles_nt + g.ct_start[c]) * g.och + k;
}

__host__ __device__ inline int pdc_lo(const PdcGeom& g, int grp) {
  return pdc_atom_at(g, (g.units * grp) / g.ngroup);
}

struct PdcTile {
  int nt, c, b, m0, i0;
};

__device__ __forceinline__ PdcTile pdc_tile(const PdcGeom& g, int t) {
  PdcTile r;
  r.nt = t / g.tiles_nt;
  const int tl = t - r.nt * g.tiles_nt;
  r.c = pdc_class(g, tl);
  const int k = tl - g.ct_start[r.c];
  r.b = k / g.tpc[r.c];
  r.m0 = (k - r.b * g.tpc[r.c]) * PD2_PIX;
  r.i0 = r.m0 / g.wc[r.c];
  return r;
}

// tap tl of class c -> (ky, kx); its G offset (dy, dx): G row = i - dy
__device__ __forceinline__ void pdc_tap(const PdcGeom& g, int c, int tl, int* ky, int* kx) {
  if (g.s == 1) {
    *ky = tl / 3;
    *kx = tl - 3 * *ky;
    return;
  }
  const int nkx = g.px[c] ? 1 : 2;
  const int a = tl / nkx, b = tl - a * nkx;
  *ky = g.py[c] ? 1 : 2 * a;
  *kx = g.px[c] ? 1 : 2 * b;
}

// loader waves (tid 0..255): staged row r = G row i0 - 1 + r (stride 1: i0 - 2 + r), staged column
// c = G column c - 1 (stride 1: c - 2); channels ch * OC ..  The thread's staged positions p = p0 +
// PPP k are the same for every atom: their (row, column) walk starts from (rc0 >> 16, rc0 & 0xFFFF)
// (one division per thread per kernel, pdc_rc0) and steps by PPP without dividing.
template <typename T, typename TG>
__device__ __forceinline__ int pdc_rc0(const PdcGeom& g, int tid) {
  constexpr int QP = PdCfg<T>::OC / PgVecP<TG>::CH;
  const int p0 = tid / QP;
  return ((p0 / g.cols) << 16) | (p0 % g.cols);
}

template <typename T, typename TG>
__device__ __forceinline__ void pdc_stage(const PdcGeom& g, T* __restrict__ dst, const TG* __restrict__ gp, int atom,
                                          int tid, int rc0) {
  typedef PgVecP<TG> PV;
  constexpr int OC = PdCfg<T>::OC, XS = PdCfg<T>::XS, CH = PV::CH, QP = OC / CH, PPP = 256 / QP;
  const int t = atom / g.och, ch = atom - t * g.och;
  const PdcTile tl = pdc_tile(g, t);
  const int r0 = tl.i0 - (g.s == 1 ? 2 : 1), c0 = g.s == 1 ? 2 : 1;
  const int npos = g.hrows * g.cols;
  const int q = tid % QP;
  const TG* src = gp + (size_t)tl.b * g.ho * g.wo * PP_O + ch * OC + CH * q;
  constexpr int U = VFD_PD_U;
  const int cstep = PPP % g.cols, rstep = PPP / g.cols;   // uniform
  int r = rc0 >> 16, c = rc0 & 0xFFFF;
  for (int p0 = tid / QP; p0 < npos; p0 += U * PPP) {
    typename PV::V v[U];
    int pos[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + PPP * u;
      const int y = r0 + r, x = c - c0;
      pos[u] = p;
      v[u] = (p < npos && y >= 0 && y < g.ho && x >= 0 && x < g.wo) ? PV::load(src + ((size_t)y * g.wo + x) * PP_O)
                                                                   : PV::zero();
      c += cstep;
      r += rstep;
      if (c >= g.cols) {
        c -= g.cols;
        ++r;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (pos[u] < npos) PV::template put<T>(dst + pos[u] * XS + CH * q, v[u]);
  }
}

// m / d for 0 <= m < 2^22, d >= 1, with rd = 1 / d: float quotient plus one correction step
__device__ __forceinline__ int pdc_div(int m, int d, float rd) {
  int q = (int)((float)m * rd);
  const int rem = m - q * d;
  q += (rem >= d) - (rem < 0);
  return q;
}

template <typename T, typename TG, typename TO = float>
__global__ __launch_bounds__(PP_THREADS, 2) void ppd_main_k(PdcGeom g, const TG* __restrict__ gp,
                                                           const void* __restrict__ Wd, TO* __restrict__ dx,
                                                           float* __restrict__ partial) {
  constexpr int OC = PdCfg<T>::OC, XS = PdCfg<T>::XS, STEPS = PdCfg<T>::STEPS, PF = PdCfg<T>::PF;
  static_assert(STEPS % PF == 0, "prefetch ring");
  constexpr bool BF = sizeof(T) == 2;
  typedef typename std::conditional<BF, bf16x8, float2>::type Frag;
  extern __shared__ __attribute__((aligned(16))) unsigned char pd_raw[];
  T* lds = reinterpret_cast<T*>(pd_raw);
  const int grp = (g.ngroup % 8 == 0) ? (blockIdx.x % 8) * (g.ngroup / 8) + blockIdx.x / 8 : blockIdx.x;
  const int a_lo = pdc_lo(g, grp), a_hi = pdc_lo(g, grp + 1);
  if (a_lo >= a_hi) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool compute = wv < PP_WAVES;
  const int rc0 = compute ? 0 : pdc_rc0<T, TG>(g, threadIdx.x - 64 * PP_WAVES);
  if (!compute) pdc_stage<T, TG>(g, lds, gp, a_lo, threadIdx.x - 64 * PP_WAVES, rc0);
  __syncthreads();
  if (!compute) {
    for (int atom = a_lo; atom < a_hi; ++atom) {
      if (atom + 1 < a_hi)
        pdc_stage<T, TG>(g, lds + ((atom + 1 - a_lo) & 1) * g.lds_elems, gp, atom + 1, threadIdx.x - 64 * PP_WAVES,
                         rc0);
      __syncthreads();
    }
    return;
  }
  const int li = lane & 31, lh = lane >> 5;
  // 2 x 2 wave grid over the 256 x 128 tile: wave (wm, wn) owns pixel blocks 4 wm .. 4 wm + 3 and
  // map-channel blocks 2 wn, 2 wn + 1 — every A fragment read from LDS feeds two MFMAs
  constexpr int MB = 4, NB = 2;
  const int wm = wv >> 1, wn = wv & 1;
  f32x16 acc[MB][NB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const Frag* wf = reinterpret_cast<const Frag*>(Wd);
  // B fragments of (atom, tap tl, step q): the weight copy's tap slot 8 - (3 ky + kx); the wave's
  // second channel block 64 fragments on
  auto bptr_t = [&](const PdcTile& tt, int ch, int tl) -> const Frag* {
    int ky, kx;
    pdc_tap(g, tt.c, tl, &ky, &kx);
    const int slot = 8 - (3 * ky + kx);
    if constexpr (BF)
      return wf + (((size_t)slot * (PP_O / 16) + ch * STEPS) * (g.np / 32) + tt.nt * (PD2_N / 32) + 2 * wn) * 64 + lane;
    else
      return wf + (((size_t)slot * (PP_O / 4) + ch * STEPS) * g.np + tt.nt * PD2_N + wn * 64 + li) * 2 + lh;
  };
  auto bptr = [&](int atom, int tl) -> const Frag* {
    const int t = atom / g.och;
    return bptr_t(pdc_tile(g, t), atom - t * g.och, tl);
  };
  const size_t qstride = BF ? (size_t)(g.np / 32) * 64 : (size_t)g.np * 2;
  Frag bq[PF][NB];
  const Frag* btap = bptr(a_lo, 0);                  // the current tap's fragments (step 0)
#pragma unroll
  for (int q = 0; q < PF; ++q)
#pragma unroll
    for (int b = 0; b < NB; ++b) bq[q][b] = btap[q * qstride + 64 * b];
  constexpr int LH = BF ? 8 : 2;
  int cur_t = -1;
  int pij[MB];                                        // (class row << 16) | class column of the lane's positions
  for (int atom = a_lo; atom < a_hi; ++atom) {
    const int t = atom / g.och, ch = atom - t * g.och;
    const PdcTile tl = pdc_tile(g, t);
    const int hw = g.hc[tl.c] * g.wc[tl.c], wcc = g.wc[tl.c];
    const int ntap = g.ntap[tl.c];
    const int rbase = tl.i0 - (g.s == 1 ? 2 : 1), cbase = g.s == 1 ? 2 : 1;
    const int m0w = tl.m0 + 32 * MB * wm;             // the wave's first position
    const float rw = 1.f / (float)wcc;
    if (t != cur_t) {                                 // position geometry once per tile (och atoms)
      cur_t = t;
#pragma unroll
      for (int a = 0; a < MB; ++a) {
        int m = m0w + 32 * a + li;
        m = m < hw ? m : hw - 1;
        const int i = pdc_div(m, wcc, rw);
        pij[a] = (i << 16) | (m - i * wcc);
      }
    }
    const T* xb = lds + ((atom - a_lo) & 1) * g.lds_elems;
    auto offsets = [&](int tp, int* o1) {
      int ky, kx;
      pdc_tap(g, tl.c, tp, &ky, &kx);
      // G row of class row i at tap ky: stride 2: i - (ky == 2) (even rows) / i (odd rows, ky = 1);
      // stride 1: Y - ky with Y = i (staged from row i0 - 2)
      const int dy = g.s == 1 ? ky : (ky == 2 ? 1 : 0), dxo = g.s == 1 ? kx : (kx == 2 ? 1 : 0);
#pragma unroll
      for (int a = 0; a < MB; ++a) {
        const int i = pij[a] >> 16, j = pij[a] & 0xFFFF;
        o1[a] = ((i - dy - rbase) * g.cols + (j - dxo + cbase)) * XS + LH * lh;
      }
    };
    int o1c[MB];
    offsets(0, o1c);
    Frag afc[MB], afn[MB];
#pragma unroll
    for (int a = 0; a < MB; ++a) afc[a] = *reinterpret_cast<const Frag*>(&xb[o1c[a]]);
    const bool more = atom + 1 < a_hi;
#pragma unroll 1
    for (int tp = 0; tp < ntap; ++tp) {
      // refill pointer: this atom's next tap, or the next atom's first
      const Frag* bn = tp + 1 < ntap ? bptr_t(tl, ch, tp + 1) : (more ? bptr(atom + 1, 0) : nullptr);
#pragma unroll
      for (int q = 0; q < STEPS; ++q) {
        if (q < STEPS - 1) {
#pragma unroll
          for (int a = 0; a < MB; ++a) afn[a] = *reinterpret_cast<const Frag*>(&xb[o1c[a] + (OC / STEPS) * (q + 1)]);
        } else if (tp + 1 < ntap) {
          offsets(tp + 1, o1c);
#pragma unroll
          for (int a = 0; a < MB; ++a) afn[a] = *reinterpret_cast<const Frag*>(&xb[o1c[a]]);
        }
#define VFD_PD_B(b) bq[q % PF][b]
        if constexpr (BF) {
#pragma unroll
          for (int a = 0; a < MB; ++a)
#pragma unroll
            for (int b = 0; b < NB; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afc[a], VFD_PD_B(b), acc[a][b], 0, 0, 0);
        } else {
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int a = 0; a < MB; ++a)
#pragma unroll
              for (int b = 0; b < NB; ++b)
                acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(s2 ? afc[a].y : afc[a].x,
                                                                 s2 ? VFD_PD_B(b).y : VFD_PD_B(b).x, acc[a][b], 0, 0, 0);
        }
#undef VFD_PD_B
        // refill the slots just read (no copy-out of the ring: see ppcb_main_k)
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          if (q + PF < STEPS)
            bq[q % PF][b] = btap[(q + PF) * qstride + 64 * b];
          else if (bn)
            bq[q % PF][b] = bn[(q + PF - STEPS) * qstride + 64 * b];
        }
#pragma unroll
        for (int a = 0; a < MB; ++a) afc[a] = afn[a];
      }
      btap = bn;
    }
    __syncthreads();                                  // buffer handed back to the loader waves
    if (ch == g.och - 1 || atom == a_hi - 1) {
      const int ts = t * g.och;
      const int n0 = tl.nt * PD2_N + wn * 64 + li;
      const int py = g.py[tl.c], px = g.px[tl.c], st = g.s;
      if (ts >= a_lo && ts + g.och <= a_hi) {         // whole tile in this range: store
        // one division per pixel block: element r sits d = (r & 3) + 8 (r >> 2) <= 27 positions
        // after the block's first, at most one class-row wrap when the class grid is >= 28 wide
        const long long rowp = (long long)st * g.wp * g.cin, colp = (long long)st * g.cin;
#pragma unroll
        for (int a = 0; a < MB; ++a) {
          const int mb = m0w + 32 * a + 4 * lh;
          const int ib = pdc_div(mb, wcc, rw), jb = mb - ib * wcc;
          TO* pa = dx + (((size_t)tl.b * g.hp + st * ib + py) * g.wp + st * jb + px) * g.cin + n0;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int d = (r & 3) + 8 * (r >> 2);
            long long off;
            if (wcc >= 28) {
              off = d * colp + (jb + d >= wcc ? rowp - wcc * colp : 0);
            } else {
              const int i2 = pdc_div(mb + d, wcc, rw), j2 = mb + d - i2 * wcc;
              off = (i2 - ib) * rowp + (j2 - jb) * colp;
            }
#pragma unroll
            for (int b = 0; b < NB; ++b) {
              if (mb + d < hw && n0 + 32 * b < g.cin) st1(pa + off + 32 * b, acc[a][b][r]);
              acc[a][b][r] = 0.f;
            }
          }
        }
      } else {
        const int slot = t == a_lo / g.och ? 0 : 1;
        float* dst = partial + ((size_t)grp * 2 + slot) * PD2_FRAG + (size_t)wv * (PD2_FRAG / PP_WAVES) + lane;
#pragma unroll
        for (int a = 0; a < MB; ++a)
#pragma unroll
          for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              dst[((a * NB + b) * 16 + r) * 64] = acc[a][b][r];
              acc[a][b][r] = 0.f;
            }
      }
    }
  }
}

template <typename TO>
__global__ __launch_bounds__(256) void ppd_reduce_k(PdcGeom g, const float* __restrict__ partial, TO* __restrict__ dx) {
  const int grp = blockIdx.x;
  const int lo = pdc_lo(g, grp);
  if (grp == 0 || lo % g.och == 0 || lo >= g.natom) return;
  const int t = lo / g.och;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c0 = (grp - 1) * 2 + (t == pdc_lo(g, grp - 1) / g.och ? 0 : 1), c1 = grp * 2;
  const PdcTile tl = pdc_tile(g, t);
  const int hw = g.hc[tl.c] * g.wc[tl.c], wcc = g.wc[tl.c];
  constexpr int FSL = 8, FPS = 8 * 16 / FSL, U = 4;
  const int contrib[2] = {c0, c1};
  // slice wv = wave (wm, wn) of ppd_main_k: fragment f = (a, b, r) -> pixel block 4 wm + a,
  // channel block 2 wn + b
  const int wm = wv >> 1, wn = wv & 1;
  for (int fu = blockIdx.y * FPS; fu < (blockIdx.y + 1) * FPS; fu += U) {
    float su[U];
    frag_sums<U>(partial, contrib, 2, PD2_FRAG, (size_t)wv * (PD2_FRAG / PP_WAVES) + (fu * 64 + lane), su);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int f = fu + u;
      const int a = f >> 5, b = (f >> 4) & 1, r = f & 15;
      const int n = tl.nt * PD2_N + wn * 64 + 32 * b + (lane & 31);
      const int m = tl.m0 + 32 * (4 * wm + a) + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (m < hw && n < g.cin) {
        const int i = m / wcc, j = m - i * wcc;
        st1(dx + (((size_t)tl.b * g.hp + g.s * i + g.py[tl.c]) * g.wp + g.s * j + g.px[tl.c]) * g.cin + n, su[u]);
      }
    }
  }
}

template <typename T>
static bool pdc_plan(const vfd_conv_desc& d, PdcGeom* out) {
  constexpr int OC = PdCfg<T>::OC, XS = PdCfg<T>::XS;
  if (d.B <= 0 || d.C <= 0 || d.C % 4 || d.stride < 1 || d.stride > 2 || d.H < 3 || d.W < 3 || d.out_channels != PP_O)
    return false;
  PdcGeom g{};
  g.B = d.B;
  g.hp = d.H;
  g.wp = d.W;
  g.cin = d.C;
  g.s = d.stride;
  g.ho = (d.H - 3) / d.stride + 1;
  g.wo = (d.W - 3) / d.stride + 1;
  if (g.ho < 1 || g.wo < 1) return false;
  g.np = (d.C + 255) / 256 * 256;
  g.ntn = (d.C + PD2_N - 1) / PD2_N;
  g.och = PP_O / OC;
  g.nclass = d.stride == 2 ? 4 : 1;
  int wmax = 0, rows_max = 0;
  g.ct_start[0] = g.cu_start[0] = 0;
  for (int c = 0; c < g.nclass; ++c) {
    g.py[c] = d.stride == 2 ? c >> 1 : 0;
    g.px[c] = d.stride == 2 ? c & 1 : 0;
    g.hc[c] = d.stride == 2 ? (d.H - g.py[c] + 1) / 2 : d.H;
    g.wc[c] = d.stride == 2 ? (d.W - g.px[c] + 1) / 2 : d.W;
    g.tpc[c] = (g.hc[c] * g.wc[c] + PD2_PIX - 1) / PD2_PIX;
    g.ntap[c] = d.stride == 2 ? (g.py[c] ? 1 : 2) * (g.px[c] ? 1 : 2) : 9;
    g.ct_start[c + 1] = g.ct_start[c] + d.B * g.tpc[c];
    g.cu_start[c + 1] = g.cu_start[c] + d.B * g.tpc[c] * g.och * g.ntap[c];
    wmax = g.wc[c] > wmax ? g.wc[c] : wmax;
    const int rows = (PD2_PIX - 1 + g.wc[c] - 1) / g.wc[c] + 1;
    rows_max = (rows < g.hc[c] ? rows : g.hc[c]) > rows_max ? (rows < g.hc[c] ? rows : g.hc[c]) : rows_max;
  }
  g.tiles_nt = g.ct_start[g.nclass];
  g.units_nt = g.cu_start[g.nclass];
  g.ntile = g.ntn * g.tiles_nt;
  g.natom = g.ntile * g.och;
  g.units = (long long)g.ntn * g.units_nt;
  // staged rows: stride 2 the tile's class rows + 1 above (ky = 2); stride 1 + 2 above
  g.hrows = rows_max + (d.stride == 1 ? 2 : 1);
  g.cols = wmax + (d.stride == 1 ? 2 : 1);
  g.lds_elems = g.hrows * g.cols * XS;
  if ((size_t)2 * g.lds_elems * sizeof(T) > PP_LDS_MAX) return false;
  // groups: every range must hold >= och atoms (a split tile meets two groups) -> units per group
  // >= max taps x och
  const int res = pp_resident();
  const long long most = g.units / (9LL * g.och);
  g.ngroup = (int)(most < res ? (most > 0 ? most : 1) : res);
  for (int k = 0; k < g.ngroup; ++k)
    if (pdc_lo(g, k + 1) - pdc_lo(g, k) < g.och && pdc_lo(g, k + 1) < g.natom) return false;
  *out = g;
  return true;
}

}  // namespace vfd

using namespace vfd;

extern "C" {

// channels per atom of the fp32 forward: 16, or 8 when 16 do not fit LDS
static int pp_cc(const vfd_conv_desc& d, PpGeom* g) {
  if (pp_plan(d, g)) return PP_CC;
  if (pp_plan(d, g, 8, 12 * 4)) return 8;
  return 0;
}

size_t vfd_pad_conv_fwd_workspace(const vfd_conv_desc* d) {
  PpGeom g;
  if (!d || !pp_cc(*d, &g)) return 0;
  return ((size_t)g.ngroup * 2 + g.ntile) * PP_FRAG * sizeof(float);
}

int vfd_pad_conv_fwd(const vfd_conv_desc* d, const float* x, const float* Wf, const float* bias, float* out,
                     void* ws, size_t ws_bytes, void* stream) {
  VFD_REQUIRE(d && x && Wf && bias && out, "pad_conv_fwd: null argument");
  PpGeom g;
  const int cc = pp_cc(*d, &g);
  VFD_REQUIRE(cc, "pad_conv_fwd: unsupported shape (C %% 4 == 0, stride 1 or 2, %d outputs, "
              "input rows of a tile in LDS)", PP_O);
  VFD_REQUIRE(ws && ws_bytes >= vfd_pad_conv_fwd_workspace(d), "pad_conv_fwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_PAD_CONV_FWD, s);
  float* partial = (float*)ws;
  if (cc == 8) {
    lds_attr(reinterpret_cast<const void*>(ppc_main_k<8>), PP_LDS_MAX);
    ppc_main_k<8><<<g.ngroup, PP_THREADS, (size_t)2 * g.lds_floats * sizeof(float), s>>>(g, x, Wf, bias, out, partial);
  } else {
    lds_attr(reinterpret_cast<const void*>(ppc_main_k<PP_CC>), PP_LDS_MAX);
    ppc_main_k<PP_CC><<<g.ngroup, PP_THREADS, (size_t)2 * g.lds_floats * sizeof(float), s>>>(g, x, Wf, bias, out,
                                                                                           partial);
  }
  ppc_reduce_k<float><<<dim3(g.ntile, PP_FSL), 256, 0, s>>>(g, partial, bias, out);
  return fail_launch("pad_conv_fwd");
}

// channels per atom of the bf16 forward: 32, or 16 when 32 do not fit LDS
static int ppb_cc(const vfd_conv_desc& d, PpGeom* g) {
  if (pp_plan(d, g, PPB_CC, PPB_XS * 2, true)) return PPB_CC;
  if (pp_plan(d, g, 16, 24 * 2, true)) return 16;
  return 0;
}

size_t vfd_pad_conv_fwd_bf16_workspace(const vfd_conv_desc* d) {
  PpGeom g;
  if (!d || !ppb_cc(*d, &g)) return 0;
  return ((size_t)g.ngroup * 2 + g.ntile) * PP_FRAG * sizeof(float);
}

int vfd_pad_conv_fwd_bf16_t(const vfd_conv_desc* d, const void* x, int dtype_x, const void* Wf, const float* bias,
                            void* out, void* ws, size_t ws_bytes, void* stream) {
  VFD_REQUIRE(d && x && Wf && bias && out, "pad_conv_fwd_bf16: null argument");
  VFD_REQUIRE(dtype_x == 0 || dtype_x == 1, "pad_conv_fwd_bf16: dtype_x %d (0 fp32, 1 bf16)", dtype_x);
  PpGeom g;
  const int cc = ppb_cc(*d, &g);
  VFD_REQUIRE(cc, "pad_conv_fwd_bf16: unsupported shape (C %% 4 == 0, stride 1 or 2, "
              "%d outputs, input rows of a tile in LDS)", PP_O);
  VFD_REQUIRE(ws && ws_bytes >= vfd_pad_conv_fwd_bf16_workspace(d), "pad_conv_fwd_bf16: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_PAD_CONV_FWD, s);
  float* partial = (float*)ws;
  const size_t lds = (size_t)2 * g.hrows * g.wp * (cc + 8) * 2;
  const bf16x8* wf = (const bf16x8*)Wf;
#define VFD_PPB_LAUNCH(CCV, TXT)                                                              \
  lds_attr(reinterpret_cast<const void*>(ppcb_main_k<CCV, TXT>), PP_LDS_MAX);                 \
  ppcb_main_k<CCV, TXT><<<g.ngroup, PP_THREADS, lds, s>>>(g, (const TXT*)x, wf, partial);
  if (cc == 16 && dtype_x == 0) {
    VFD_PPB_LAUNCH(16, float)
  } else if (cc == 16) {
    VFD_PPB_LAUNCH(16, __bf16)
  } else if (dtype_x == 0) {
    VFD_PPB_LAUNCH(PPB_CC, float)
  } else {
    VFD_PPB_LAUNCH(PPB_CC, __bf16)
  }
#undef VFD_PPB_LAUNCH
  ppc_reduce_k<__bf16><<<dim3(g.ntile, PP_FSL), 256, 0, s>>>(g, partial, bias, (__bf16*)out);
  return fail_launch("pad_conv_fwd_bf16");
}

int vfd_pad_conv_fwd_bf16(const vfd_conv_desc* d, const float* x, const void* Wf, const float* bias, void* out,
                          void* ws, size_t ws_bytes, void* stream) {
  return vfd_pad_conv_fwd_bf16_t(d, x, 0, Wf, bias, out, ws, ws_bytes, stream);
}

size_t vfd_pad_conv_dgrad_workspace(const vfd_conv_desc* d) {
  PdcGeom g;
  if (!d || !pdc_plan<float>(*d, &g)) return 0;
  return (size_t)g.ngroup * 2 * PD2_FRAG * sizeof(float);
}

int vfd_pad_conv_dgrad(const vfd_conv_desc* d, const float* g_pre, const float* Wd, float* dx, void* ws,
                       size_t ws_bytes, void* stream) {
  VFD_REQUIRE(d && g_pre && Wd && dx, "pad_conv_dgrad: null argument");
  PdcGeom g;
  VFD_REQUIRE(pdc_plan<float>(*d, &g), "pad_conv_dgrad: unsupported shape (C %% 4 == 0, stride 1 or 2, %d outputs)", PP_O);
  VFD_REQUIRE(ws && ws_bytes >= vfd_pad_conv_dgrad_workspace(d), "pad_conv_dgrad: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_PAD_CONV_DGRAD, s);
  lds_attr(reinterpret_cast<const void*>(ppd_main_k<float, float>), PP_LDS_MAX);
  ppd_main_k<float, float><<<g.ngroup, PP_THREADS, (size_t)2 * g.lds_elems * sizeof(float), s>>>(g, g_pre, Wd, dx,
                                                                                                 (float*)ws);
  ppd_reduce_k<float><<<dim3(g.ngroup, 8), 256, 0, s>>>(g, (const float*)ws, dx);
  return fail_launch("pad_conv_dgrad");
}

size_t vfd_pad_conv_dgrad_bf16_workspace(const vfd_conv_desc* d) {
  PdcGeom g;
  if (!d || !pdc_plan<__bf16>(*d, &g)) return 0;
  return (size_t)g.ngroup * 2 * PD2_FRAG * sizeof(float);
}

// dtype_dx 0: fp32 d X, 1: bf16 (rounded once from the fp32 sums, as a bf16 conv's input gradient)
int vfd_pad_conv_dgrad_bf16_t(const vfd_conv_desc* d, const void* g_pre, const void* Wd, void* dx, int dtype_dx,
                              void* ws, size_t ws_bytes, void* stream) {
  VFD_REQUIRE(d && g_pre && Wd && dx && (dtype_dx == 0 || dtype_dx == 1), "pad_conv_dgrad_bf16: bad argument");
  PdcGeom g;
  VFD_REQUIRE(pdc_plan<__bf16>(*d, &g), "pad_conv_dgrad_bf16: unsupported shape (C %% 4 == 0, stride 1 or 2, %d outputs)",
              PP_O);
  VFD_REQUIRE(ws && ws_bytes >= vfd_pad_conv_dgrad_bf16_workspace(d), "pad_conv_dgrad_bf16: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_PAD_CONV_DGRAD, s);
  const size_t lds = (size_t)2 * g.lds_elems * sizeof(__bf16);
  if (dtype_dx == 1) {
    lds_attr(reinterpret_cast<const void*>(ppd_main_k<__bf16, __bf16, __bf16>), PP_LDS_MAX);
    ppd_main_k<__bf16, __bf16, __bf16><<<g.ngroup, PP_THREADS, lds, s>>>(g, (const __bf16*)g_pre, Wd, (__bf16*)dx,
                                                                         (float*)ws);
    ppd_reduce_k<__bf16><<<dim3(g.ngroup, 8), 256, 0, s>>>(g, (const float*)ws, (__bf16*)dx);
  } else {
    lds_attr(reinterpret_cast<const void*>(ppd_main_k<__bf16, __bf16, float>), PP_LDS_MAX);
    ppd_main_k<__bf16, __bf16, float><<<g.ngroup, PP_THREADS, lds, s>>>(g, (const __bf16*)g_pre, Wd, (float*)dx,
                                                                        (float*)ws);
    ppd_reduce_k<float><<<dim3(g.ngroup, 8), 256, 0, s>>>(g, (const float*)ws, (float*)dx);
  }
  return fail_launch("pad_conv_dgrad_bf16");
}

int vfd_pad_conv_dgrad_bf16(const vfd_conv_desc* d, const void* g_pre, const void* Wd, float* dx, void* ws,
                            size_t ws_bytes, void* stream) {
  return vfd_pad_conv_dgrad_bf16_t(d, g_pre, Wd, dx, 0, ws, ws_bytes, stream);
}

}  // extern "C"
