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

struct PpGeom {
  int B, hp, wp, cin, s, ho, wo, mimg, mtiles, nchunk, cq, ntile, natom, ngroup, hrows, lds_floats;
};

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
// ch*16 .. ch*16 + 15 (zero past Cin)
__device__ __forceinline__ void pp_stage(const PpGeom& g, float* __restrict__ dst, const float* __restrict__ x,
                                         int atom, int tid) {
  const int t = atom / g.nchunk, ch = atom - t * g.nchunk;
  const PpTile tl = pp_tile(g, t);
  const int npos = g.hrows * g.wp;
  const int q = tid & 3;
  const int c = ch * PP_CC + 4 * q;
  const int r0 = g.s * tl.ymin;
  const float* src = x + ((size_t)tl.b * g.hp + r0) * g.wp * g.cin + c;
  const bool cok = c < g.cin;
  for (int p0 = tid >> 2; p0 < npos; p0 += 4 * 64) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = p0 + 64 * u;
      v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (cok && p < npos && r0 + p / g.wp < g.hp)
        v[u] = *reinterpret_cast<const float4*>(src + (size_t)p * g.cin);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = p0 + 64 * u;
      if (p < npos) *reinterpret_cast<float4*>(dst + p * PP_XS + 4 * q) = v[u];
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
// (channels past Cin zero).
__global__ __launch_bounds__(PP_THREADS, 2) void ppc_main_k(PpGeom g, const float* __restrict__ x,
                                                           const float* __restrict__ Wf,
                                                           const float* __restrict__ bias,
                                                           float* __restrict__ out,
                                                           float* __restrict__ partial) {
  extern __shared__ float pp_lds[];
  const int grp = blockIdx.x;
  const int a_lo = pp_lo(g, grp), a_hi = pp_lo(g, grp + 1);
  if (a_lo >= a_hi) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool compute = wv < PP_WAVES;
  if (!compute) pp_stage(g, pp_lds, x, a_lo, threadIdx.x - 64 * PP_WAVES);
  __syncthreads();
  if (!compute) {
    for (int atom = a_lo; atom < a_hi; ++atom) {
      if (atom + 1 < a_hi)
        pp_stage(g, pp_lds + ((atom + 1 - a_lo) & 1) * g.lds_floats, x, atom + 1, threadIdx.x - 64 * PP_WAVES);
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
  float2 bq[PP_PF][2];
  int pf_atom = a_lo, pf_it = 0;
  auto prefetch = [&](int slot) {
    if (pf_atom < a_hi) {
      const int ch = pf_atom % g.nchunk;
      const int tap = pf_it >> 2, q = pf_it & 3;
      const float2* w = wlane + (size_t)(tap * g.cq + ch * (PP_CC / 4) + q) * (2 * PP_O);
      bq[slot][0] = w[0];
      bq[slot][1] = w[64];
      if (++pf_it == PP_ITERS) { pf_it = 0; ++pf_atom; }
    }
  };
#pragma unroll
  for (int k = 0; k < PP_PF; ++k) prefetch(k);
  for (int atom = a_lo; atom < a_hi; ++atom) {
    const int t = atom / g.nchunk, ch = atom - t * g.nchunk;
    const PpTile tl = pp_tile(g, t);
    int aoff[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      int m = tl.m0 + 32 * a + li;
      m = m < g.mimg ? m : g.mimg - 1;                 // pixels past the image: computed, never stored
      const int y = m / g.wo, xx = m - y * g.wo;
      aoff[a] = (g.s * (y - tl.ymin) * g.wp + g.s * xx) * PP_XS + 2 * lh;
    }
    const float* xb = pp_lds + ((atom - a_lo) & 1) * g.lds_floats;
    float2 afc[4], afn[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) afc[a] = *reinterpret_cast<const float2*>(&xb[aoff[a]]);
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap - 3 * ky;
      const float* xt = xb + (ky * g.wp + kx) * PP_XS;
      const int tn = tap + 1, kyn = tn / 3, kxn = tn - 3 * kyn;
      const float* xn = xb + (kyn * g.wp + kxn) * PP_XS;
#pragma unroll
      for (int q = 0; q < PP_CC / 4; ++q) {
        const int ring = q % PP_PF;
        const float2 b0 = bq[ring][0], b1 = bq[ring][1];
        prefetch(ring);
        if (q < PP_CC / 4 - 1) {
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
constexpr int PPB_CC = 32;                      // input channels per atom
constexpr int PPB_XS = PPB_CC + 8;              // bf16 per staged position (80 B: 16-B aligned)
constexpr int PPB_STEPS = 9 * (PPB_CC / 16);    // (tap, 16-channel) MFMA steps per atom
constexpr int PPB_PF = 2;                       // weight-fragment prefetch distance (steps)

__device__ __forceinline__ void ppb_stage(const PpGeom& g, __bf16* __restrict__ dst, const float* __restrict__ x,
                                          int atom, int tid) {
  const int nchunk = (g.cin + PPB_CC - 1) / PPB_CC;
  const int t = atom / nchunk, ch = atom - t * nchunk;
  const PpTile tl = pp_tile(g, t);
  const int npos = g.hrows * g.wp;
  const int q = tid & 7;                        // channel quad of the 32-channel chunk
  const int c = ch * PPB_CC + 4 * q;
  const int r0 = g.s * tl.ymin;
  const float* src = x + ((size_t)tl.b * g.hp + r0) * g.wp * g.cin + c;
  const bool cok = c < g.cin;                   // cin % 4 == 0: a quad is all in or all out
  for (int p0 = tid >> 3; p0 < npos; p0 += 4 * 32) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = p0 + 32 * u;
      v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (cok && p < npos && r0 + p / g.wp < g.hp)
        v[u] = *reinterpret_cast<const float4*>(src + (size_t)p * g.cin);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = p0 + 32 * u;
      if (p < npos) {
        bf16x4 b;
        b[0] = (__bf16)v[u].x;
        b[1] = (__bf16)v[u].y;
        b[2] = (__bf16)v[u].z;
        b[3] = (__bf16)v[u].w;
        *reinterpret_cast<bf16x4*>(dst + p * PPB_XS + 4 * q) = b;
      }
    }
  }
}

__global__ __launch_bounds__(PP_THREADS, 2) void ppcb_main_k(PpGeom g, const float* __restrict__ x,
                                                            const bf16x8* __restrict__ Wf,
                                                            float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) __bf16 ppb_lds[];
  const int grp = blockIdx.x;
  const int a_lo = pp_lo(g, grp), a_hi = pp_lo(g, grp + 1);
  if (a_lo >= a_hi) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool compute = wv < PP_WAVES;
  const int lds_elems = g.hrows * g.wp * PPB_XS;
  if (!compute) ppb_stage(g, ppb_lds, x, a_lo, threadIdx.x - 64 * PP_WAVES);
  __syncthreads();
  if (!compute) {
    for (int atom = a_lo; atom < a_hi; ++atom) {
      if (atom + 1 < a_hi)
        ppb_stage(g, ppb_lds + ((atom + 1 - a_lo) & 1) * lds_elems, x, atom + 1, threadIdx.x - 64 * PP_WAVES);
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
  const int nchunk = g.nchunk;                  // 32-channel chunks (host-set for the bf16 form)
  const int nq16 = nchunk * (PPB_CC / 16);
  const bf16x8* wlane = Wf + (size_t)(2 * wv) * 64 + lane;
  bf16x8 bq[PPB_PF][2];
  int pf_atom = a_lo, pf_it = 0;
  auto prefetch = [&](int slot) {
    if (pf_atom < a_hi) {
      const int ch = pf_atom % nchunk;
      const int tap = pf_it >> 1, q = pf_it & 1;
      const bf16x8* w = wlane + ((size_t)tap * nq16 + ch * (PPB_CC / 16) + q) * (PP_O / 32) * 64;
      bq[slot][0] = w[0];
      bq[slot][1] = w[64];
      if (++pf_it == PPB_STEPS) { pf_it = 0; ++pf_atom; }
    }
  };
#pragma unroll
  for (int k = 0; k < PPB_PF; ++k) prefetch(k);
  for (int atom = a_lo; atom < a_hi; ++atom) {
    const int t = atom / nchunk, ch = atom - t * nchunk;
    const PpTile tl = pp_tile(g, t);
    int aoff[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      int m = tl.m0 + 32 * a + li;
      m = m < g.mimg ? m : g.mimg - 1;                 // pixels past the image: computed, never stored
      const int y = m / g.wo, xx = m - y * g.wo;
      aoff[a] = (g.s * (y - tl.ymin) * g.wp + g.s * xx) * PPB_XS + 8 * lh;
    }
    const __bf16* xb = ppb_lds + ((atom - a_lo) & 1) * lds_elems;
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap - 3 * ky;
      const __bf16* xt = xb + (ky * g.wp + kx) * PPB_XS;
#pragma unroll
      for (int q = 0; q < PPB_CC / 16; ++q) {
        bf16x8 af[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) af[a] = *reinterpret_cast<const bf16x8*>(&xt[aoff[a] + 16 * q]);
        const int ring = q % PPB_PF;
        const bf16x8 b0 = bq[ring][0], b1 = bq[ring][1];
        prefetch(ring);
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          acc[a][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], b0, acc[a][0], 0, 0, 0);
          acc[a][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], b1, acc[a][1], 0, 0, 0);
        }
      }
    }
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

static bool pp_plan(const vfd_conv_desc& d, PpGeom* out, int cc = PP_CC, int xs_bytes = PP_XS * 4) {
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
  g.cq = g.nchunk * (cc / 4);
  g.ntile = g.B * g.mtiles;
  g.natom = g.ntile * g.nchunk;
  // output rows under 128 consecutive pixels, and the input rows they read
  const int orows = 1 + (g.wo - 1 + PP_PIX - 1) / g.wo;
  g.hrows = g.s * (orows - 1) + 3;
  g.lds_floats = g.hrows * g.wp * PP_XS;
  if ((size_t)2 * g.hrows * g.wp * xs_bytes > PP_LDS_MAX) return false;
  // ranges of >= ceil(nchunk / (PP_MAXC - 2)) atoms keep a tile's contributors <= PP_MAXC - 1
  const int res = pp_resident();
  const int min_range = (g.nchunk + PP_MAXC - 3) / (PP_MAXC - 2);
  int most = g.natom / min_range;
  most = most > 0 ? most : 1;
  g.ngroup = res < most ? res : most;
  *out = g;
  return true;
}

}  // namespace vfd

using namespace vfd;

extern "C" {

size_t vfd_pad_conv_fwd_workspace(const vfd_conv_desc* d) {
  PpGeom g;
  if (!d || !pp_plan(*d, &g)) return 0;
  return ((size_t)g.ngroup * 2 + g.ntile) * PP_FRAG * sizeof(float);
}

int vfd_pad_conv_fwd(const vfd_conv_desc* d, const float* x, const float* Wf, const float* bias, float* out,
                     void* ws, size_t ws_bytes, void* stream) {
  VFD_REQUIRE(d && x && Wf && bias && out, "pad_conv_fwd: null argument");
  PpGeom g;
  VFD_REQUIRE(pp_plan(*d, &g), "pad_conv_fwd: unsupported shape (C %% 4 == 0, stride 1 or 2, %d outputs, "
              "input rows of a tile in LDS)", PP_O);
  VFD_REQUIRE(ws && ws_bytes >= vfd_pad_conv_fwd_workspace(d), "pad_conv_fwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_PAD_CONV_FWD, s);
  lds_attr(reinterpret_cast<const void*>(ppc_main_k), PP_LDS_MAX);
  float* partial = (float*)ws;
  ppc_main_k<<<g.ngroup, PP_THREADS, (size_t)2 * g.lds_floats * sizeof(float), s>>>(g, x, Wf, bias, out, partial);
  ppc_reduce_k<float><<<dim3(g.ntile, PP_FSL), 256, 0, s>>>(g, partial, bias, out);
  return fail_launch("pad_conv_fwd");
}

size_t vfd_pad_conv_fwd_bf16_workspace(const vfd_conv_desc* d) {
  PpGeom g;
  if (!d || !pp_plan(*d, &g, PPB_CC, PPB_XS * 2)) return 0;
  return ((size_t)g.ngroup * 2 + g.ntile) * PP_FRAG * sizeof(float);
}

int vfd_pad_conv_fwd_bf16(const vfd_conv_desc* d, const float* x, const void* Wf, const float* bias, void* out,
                          void* ws, size_t ws_bytes, void* stream) {
  VFD_REQUIRE(d && x && Wf && bias && out, "pad_conv_fwd_bf16: null argument");
  PpGeom g;
  VFD_REQUIRE(pp_plan(*d, &g, PPB_CC, PPB_XS * 2), "pad_conv_fwd_bf16: unsupported shape (C %% 4 == 0, stride 1 or 2, "
              "%d outputs, input rows of a tile in LDS)", PP_O);
  VFD_REQUIRE(ws && ws_bytes >= vfd_pad_conv_fwd_bf16_workspace(d), "pad_conv_fwd_bf16: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_PAD_CONV_FWD, s);
  lds_attr(reinterpret_cast<const void*>(ppcb_main_k), PP_LDS_MAX);
  float* partial = (float*)ws;
  const size_t lds = (size_t)2 * g.hrows * g.wp * PPB_XS * 2;
  ppcb_main_k<<<g.ngroup, PP_THREADS, lds, s>>>(g, x, (const bf16x8*)Wf, partial);
  ppc_reduce_k<__bf16><<<dim3(g.ntile, PP_FSL), 256, 0, s>>>(g, partial, bias, (__bf16*)out);
  return fail_launch("pad_conv_fwd_bf16");
}

}  // extern "C"
