// Weight relayouts for the MFMA convolution kernels (once per step: the weights change at every
// optimizer step).  Each replaces a chain of ATen permute / flip / pad / contiguous copies whose
// element-wise gathers touch every 3x3 tap row of the source once per tap (~0.6 TB/s on the
// 47 MB pose reduce_dim weight):  here a thread moves one (out-channel, in-channel) row of the 9
// taps — a 36-byte contiguous read — to the 9 tap planes of the destination, where consecutive
// lanes write consecutive floats.
//
//   mode 0  K2C fragments           dst[tap][q][o][h][s]     = w[o][chan(4q + 2h + s)][tap]
//           (padconv.hip ppc_main_k; cz = 4q + 2h + s in the map's channel order, zero past C;
//           chan(cz) = cz, or for the pose map's z-major order cz = z*C1 + c the reference
//           channel c*Z + z — volumetric_fusionnet.py:160-162, 338-343)
//   mode 1  K3C forward fragments   dst[d][tap][q][o][h][s]  = w[o][(4q + 2h + s)*D + d][tap]
//           (projconv.hip pcv_main_k; reference channel c*D + d, :261-265)
//   mode 2  K3C data-gradient copy  dst[8 - tap][oq][n][h][s] = w[4oq + 2h + s][c*D + d][tap]
//           (projconv.hip pcd_main_k; n = d*Cv + c, zero for n >= Cv*D)
//   mode 3  K3C forward, bf16       dst[d][tap][q16][ob][lane][j] = bf16(w[o][c*D + d][tap]),
//           o = 32 ob + (lane & 31), c = 16 q16 + 8 (lane >> 5) + j (projconv.hip pcvb_main_k)
//   mode 4  K2C, bf16 (from the mode-0 copy f0): dst[tap][q16][ob][lane][j] = bf16(f0 of channel
//           16 q16 + 8 (lane >> 5) + j, out-channel 32 ob + (lane & 31)), q16 < ceil32(C) / 16
//   mode 5  K3C data gradient, bf16 (from the mode-2 copy f2): dst[tap'][q16][nb][lane][j] = bf16(f2 of
//           out-channel 16 q16 + 8 (lane >> 5) + j, n = 32 nb + (lane & 31)) (projconv.hip pcg_main_k)
//   permute element (o, a, b, t) between any two strided layouts (the pose weight between the
//           reference channel order c*Z + z and the map's z*C1 + c, NCHW or channels-last for MIOpen);
//           swap = the NCHW -> NCHW instance dst[o][b][a][t] = w[o][a][b][t]
#include "vfd_common.h"

namespace vfd {

constexpr int WR_TAPS = 9;

struct WrArgs {
  int mode, O, C, C1, Z, Cv, D, cpad, npad, refperm;
};

__global__ __launch_bounds__(256) void weight_frag_k(WrArgs a, const float* __restrict__ w, float* __restrict__ dst,
                                                     long long nrow) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;   // destination row (all taps)
  if (t >= nrow) return;
  const int s = (int)(t & 1), h = (int)((t >> 1) & 1);
  long long src = -1;                     // source row (of 9 taps), -1: zero padding
  long long plane = 0, off = 0;           // tap-plane stride, offset of tap 0 in dst
  int flip = 0;
  const int K = a.mode == 0 ? a.C : a.Cv * a.D;   // source in-channels per out-channel
  if (a.mode == 0) {
    const long long per = (long long)(a.cpad / 4) * a.O * 4;             // one tap plane
    const int o = (int)((t >> 2) % a.O), q = (int)((t >> 2) / a.O);
    const int cz = 4 * q + 2 * h + s;
    if (cz < a.C) src = (long long)o * K + (a.refperm ? (long long)(cz % a.C1) * a.Z + cz / a.C1 : cz);
    plane = per;
    off = t;
  } else if (a.mode == 1) {
    const int Q = a.Cv / 4;
    const long long per = (long long)Q * a.O * 4;
    const long long r = t % per;
    const int d = (int)(t / per);
    const int o = (int)((r >> 2) % a.O), q = (int)((r >> 2) / a.O);
    const int c = 4 * q + 2 * h + s;
    src = (long long)o * K + (long long)c * a.D + d;
    plane = per;
    off = (long long)d * WR_TAPS * per + r;
  } else {
    const long long per = (long long)(a.O / 4) * a.npad * 4;
    const int n = (int)((t >> 2) % a.npad), oq = (int)((t >> 2) / a.npad);
    const int o = 4 * oq + 2 * h + s;
    if (n < K) src = (long long)o * K + (long long)(n % a.Cv) * a.D + n / a.Cv;
    plane = per;
    off = t;
    flip = 1;
  }
  float v[WR_TAPS];
  const float* p = w + (src >= 0 ? src : 0) * WR_TAPS;
#pragma unroll
  for (int k = 0; k < WR_TAPS; ++k) v[k] = src >= 0 ? p[k] : 0.f;
#pragma unroll
  for (int k = 0; k < WR_TAPS; ++k) dst[off + (flip ? WR_TAPS - 1 - k : k) * plane] = v[k];
}

// Tiled forms of the three fragment modes for the step's large weights: a workgroup stages a
// tile whose source rows are contiguous runs (a 9-tap row per (out, in)-channel, several rows in
// a run) through LDS, then writes destination runs of 32-64 consecutive floats.  Same values and
// placement as weight_frag_k (a copy: bit-identical); weight_frag_k stays for shapes the tiles do
// not cover.
constexpr int WT_DT = 10;                 // depth bins per tile (modes 1, 2)
constexpr int WT_TILE = 64 * WT_DT * WR_TAPS;

// mode 1: tile = 16 out-channels x one channel quad q x WT_DT depth bins; source runs
// w[o][(4q + c) * D + d0 .. + nd][taps] (nd * 9 floats), destination runs (d, tap, q): 16 o x 4 c
__global__ __launch_bounds__(256) void wfrag1_k(const float* __restrict__ w, float* __restrict__ dst, int O, int Cv,
                                                int D) {
  __shared__ float tile[WT_TILE];
  const int o0 = blockIdx.x * 16, q = blockIdx.y, d0 = blockIdx.z * WT_DT;
  const int nd = min(WT_DT, D - d0), K = Cv * D, Q = Cv / 4;
  const int seg = nd * WR_TAPS, no = min(16, O - o0);
  for (int i = threadIdx.x; i < 64 * seg; i += 256) {
    const int r = i / seg, k = i - r * seg;          // r = o_l * 4 + c_l
    if ((r >> 2) < no)
      tile[r * WT_DT * WR_TAPS + k] = w[((size_t)(o0 + (r >> 2)) * K + (size_t)(4 * q + (r & 3)) * D + d0) * WR_TAPS + k];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < seg * 64; i += 256) {
    const int r = i & 63, dt = i >> 6;               // dt = d_l * 9 + tap
    const int d_l = dt / WR_TAPS, tap = dt - d_l * WR_TAPS;
    if ((r >> 2) < no)
      dst[(((size_t)(d0 + d_l) * WR_TAPS + tap) * Q + q) * O * 4 + (size_t)o0 * 4 + r] = tile[r * WT_DT * WR_TAPS + dt];
  }
}

// mode 2: tile = one out-channel quad oq x 16 channels x WT_DT depth bins; source runs
// w[4 oq + o][(c0 + c) * D + d0 .. + nd][taps], destination runs (8 - tap, oq, d): 16 c x 4 o
// (n = d * Cv + c); the zero rows n >= Cv * D are written by wfrag2_pad_k
__global__ __launch_bounds__(256) void wfrag2_k(const float* __restrict__ w, float* __restrict__ dst, int O, int Cv,
                                                int D, int npad) {
  __shared__ float tile[WT_TILE];
  const int oq = blockIdx.x, c0 = blockIdx.y * 16, d0 = blockIdx.z * WT_DT;
  const int nd = min(WT_DT, D - d0), K = Cv * D, OQ = O / 4;
  const int seg = nd * WR_TAPS, nc = min(16, Cv - c0);
  for (int i = threadIdx.x; i < 64 * seg; i += 256) {
    const int r = i / seg, k = i - r * seg;          // r = o_l * 16 + c_l
    const int o_l = r >> 4, c_l = r & 15;
    if (c_l < nc)
      tile[r * WT_DT * WR_TAPS + k] = w[((size_t)(4 * oq + o_l) * K + (size_t)(c0 + c_l) * D + d0) * WR_TAPS + k];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < seg * 64; i += 256) {
    const int r = i & 63, dt = i >> 6;
    const int c_l = r >> 2, o_l = r & 3;
    const int d_l = dt / WR_TAPS, tap = dt - d_l * WR_TAPS;
    if (c_l < nc) {
      const size_t n = (size_t)(d0 + d_l) * Cv + c0 + c_l;
      dst[(((size_t)(WR_TAPS - 1 - tap) * OQ + oq) * npad + n) * 4 + o_l] = tile[(o_l * 16 + c_l) * WT_DT * WR_TAPS + dt];
    }
  }
}

__global__ __launch_bounds__(256) void wfrag2_pad_k(float* __restrict__ dst, int OQ, int K, int npad) {
  const long long per = (long long)(npad - K) * 4;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)WR_TAPS * OQ * per) return;
  const long long plane = i / per, r = i - plane * per;    // plane = tap' * OQ + oq
  dst[(plane * npad + K) * 4 + r] = 0.f;
}

// mode 3 (bf16, projconv.hip pcvb_main_k): dst[d][tap][q16][ob][lane][j] = bf16(w[o][c*D + d][tap])
// with o = 32 ob + (lane & 31), c = 16 q16 + 8 (lane >> 5) + j (round to nearest even).  Tile = one
// 32-out-channel block x one 16-channel chunk x WT_D3 depth bins, source runs of WT_D3 * 9 floats
// staged through LDS; each thread writes one lane's 16-B fragment.
constexpr int WT_D3 = 4;
typedef __bf16 wbf16x8 __attribute__((ext_vector_type(8)));
__global__ __launch_bounds__(256) void wfrag3_k(const float* __restrict__ w, wbf16x8* __restrict__ dst, int O, int Cv,
                                                int D) {
  __shared__ float tile[32 * 16 * WT_D3 * WR_TAPS];
  const int ob = blockIdx.x, q16 = blockIdx.y, d0 = blockIdx.z * WT_D3;
  const int nd = min(WT_D3, D - d0), K = Cv * D, seg = nd * WR_TAPS;
  for (int i = threadIdx.x; i < 32 * 16 * seg; i += 256) {
    const int r = i / seg, k = i - r * seg;          // r = o_l * 16 + c_l
    const int o_l = r >> 4, c_l = r & 15;
    tile[r * WT_D3 * WR_TAPS + k] = w[((size_t)(32 * ob + o_l) * K + (size_t)(16 * q16 + c_l) * D + d0) * WR_TAPS + k];
  }
  __syncthreads();
  const int Q16 = Cv / 16, OB = O / 32;
  for (int i = threadIdx.x; i < seg * 64; i += 256) {
    const int lane = i & 63, dt = i >> 6;            // dt = d_l * 9 + tap
    const int d_l = dt / WR_TAPS, tap = dt - d_l * WR_TAPS;
    const int o_l = lane & 31, h = lane >> 5;
    wbf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (__bf16)tile[(o_l * 16 + 8 * h + j) * WT_D3 * WR_TAPS + dt];
    dst[((((size_t)(d0 + d_l) * WR_TAPS + tap) * Q16 + q16) * OB + ob) * 64 + lane] = v;
  }
}

// mode 4 (bf16, padconv.hip ppcb_main_k) from the fp32 mode-0 fragment copy f0 [9][cpad16/4][O][2][2]:
// dst[tap][q16][ob][lane][j] = bf16(f0 element of channel cz = 16 q16 + 8 (lane >> 5) + j, out-channel
// 32 ob + (lane & 31)), zero for cz >= cpad16; one thread per destination lane fragment: two
// 16-B reads (channel quads 4 q16 + 2h, +1), coalesced over the 32 out-channels of a block
__global__ __launch_bounds__(256) void wfrag4_k(const float4* __restrict__ f0, wbf16x8* __restrict__ dst, int O,
                                                int cq4, int nq16) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int OB = O / 32;
  const long long total = (long long)WR_TAPS * nq16 * OB * 64;
  if (i >= total) return;
  const int lane = (int)(i & 63);
  long long r = i >> 6;
  const int ob = (int)(r % OB);
  r /= OB;
  const int q16 = (int)(r % nq16), tap = (int)(r / nq16);
  const int o = 32 * ob + (lane & 31), h = lane >> 5;
  wbf16x8 v;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q4 = 4 * q16 + 2 * h + k;
    float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
    if (q4 < cq4) f = f0[((size_t)tap * cq4 + q4) * O + o];
    v[4 * k + 0] = (__bf16)f.x;
    v[4 * k + 1] = (__bf16)f.y;
    v[4 * k + 2] = (__bf16)f.z;
    v[4 * k + 3] = (__bf16)f.w;
  }
  dst[i] = v;
}

// mode 5 (bf16, projconv.hip pcg_main_k<bf16>) from the fp32 mode-2 copy f2 [9][O/4][npad][2][2]:
// dst[tap'][q16][nb][lane][j] = bf16(f2 element of out-channel o = 16 q16 + 8 (lane >> 5) + j, n = 32 nb +
// (lane & 31)); one thread per destination lane fragment: two 16-B reads (out-channel quads
// 4 q16 + 2h, +1), coalesced over the 32 n of a block
__global__ __launch_bounds__(256) void wfrag5_k(const float4* __restrict__ f2, wbf16x8* __restrict__ dst, int OQ,
                                                int npad) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int NB = npad / 32, Q16 = OQ / 4;
  const long long total = (long long)WR_TAPS * Q16 * NB * 64;
  if (i >= total) return;
  const int lane = (int)(i & 63);
  long long r = i >> 6;
  const int nb = (int)(r % NB);
  r /= NB;
  const int q16 = (int)(r % Q16), tap = (int)(r / Q16);
  const int n = 32 * nb + (lane & 31), h = lane >> 5;
  wbf16x8 v;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float4 f = f2[((size_t)tap * OQ + 4 * q16 + 2 * h + k) * npad + n];
    v[4 * k + 0] = (__bf16)f.x;
    v[4 * k + 1] = (__bf16)f.y;
    v[4 * k + 2] = (__bf16)f.z;
    v[4 * k + 3] = (__bf16)f.w;
  }
  dst[i] = v;
}

// mode 0 with the pose map's channel order (cz = z * C1 + c, reference channel c * Z + z):
// tile = 8 out-channels x 4 map channels c0 .. c0 + 3 x all Z; source runs w[o][c0 * Z .. (c0 + 4) * Z][taps]
// (4 Z rows), destination runs (tap, q = (z C1 + c0) / 4): 8 o x 4 cz.  Needs C1 % 4 == 0 and
// C1 * Z % 16 == 0 (no zero rows).  Dynamic LDS: 8 * 4 * Z * 9 floats.
__global__ __launch_bounds__(256) void wfrag0z_k(const float* __restrict__ w, float* __restrict__ dst, int O, int C1,
                                                 int Z) {
  extern __shared__ float wt_sm[];
  const int o0 = blockIdx.x * 8, c0 = blockIdx.y * 4;
  const int C = C1 * Z, seg = 4 * Z * WR_TAPS, no = min(8, O - o0);
  for (int i = threadIdx.x; i < 8 * seg; i += 256) {
    const int o_l = i / seg, k = i - o_l * seg;
    if (o_l < no) wt_sm[i] = w[((size_t)(o0 + o_l) * C + (size_t)c0 * Z) * WR_TAPS + k];
  }
  __syncthreads();
  const int qn = C / 4;
  for (int i = threadIdx.x; i < Z * WR_TAPS * 32; i += 256) {
    const int r = i & 31, zt = i >> 5;
    const int o_l = r >> 2, c_l = r & 3;
    const int z = zt / WR_TAPS, tap = zt - z * WR_TAPS;
    if (o_l < no) {
      const int q = (z * C1 + c0) >> 2;
      dst[(((size_t)tap * qn + q) * O + o0 + o_l) * 4 + c_l] = wt_sm[o_l * seg + ((c_l * Z) + z) * WR_TAPS + tap];
    }
  }
}

// Generic 4-D permuted copy of a weight, element (o, a, b, t) from src[o so + a sa + b sb + t st]
// to dst[o do + a da + b db + t dt] (t <= 9 taps): tiles of 16 x 16 (a, b) x all taps go through
// LDS so that whichever of a / b is contiguous on either side is walked by consecutive lanes.
// The pose weight's channel-order swap (reference c*Z + z <-> K2's map order z*C1 + c) and its
// NCHW <-> channels-last conversions for MIOpen are instances.
constexpr int WS_T = 16;
struct WpArgs {
  long long so, sa, sb, st, dO, da, db, dt;
  int O, A, B, T, tiles_b;
};
__global__ __launch_bounds__(256) void weight_permute_k(WpArgs p, const float* __restrict__ w, float* __restrict__ dst) {
  __shared__ float tile[WS_T * WS_T * WR_TAPS + WS_T];
  const int o = blockIdx.y;
  const int a0 = (blockIdx.x / p.tiles_b) * WS_T, b0 = (blockIdx.x % p.tiles_b) * WS_T;
  const int t = threadIdx.x;
  const int n = WS_T * WS_T * p.T;
  // read order: the faster-moving of a / b on the source side fastest (after t if t is contiguous)
  const bool b_fast_src = p.sb <= p.sa;
  for (int k = t; k < n; k += 256) {
    int al, bl, tp;
    if (p.st == 1) {
      tp = k % p.T;
      const int r = k / p.T;
      if (b_fast_src) { bl = r % WS_T; al = r / WS_T; } else { al = r % WS_T; bl = r / WS_T; }
    } else {
      const int r = k % (WS_T * WS_T);
      tp = k / (WS_T * WS_T);
      if (b_fast_src) { bl = r % WS_T; al = r / WS_T; } else { al = r % WS_T; bl = r / WS_T; }
    }
    const int a = a0 + al, b = b0 + bl;
    if (a < p.A && b < p.B)
      tile[(al * WS_T + bl) * WR_TAPS + tp] = w[o * p.so + a * p.sa + b * p.sb + tp * p.st];
  }
  __syncthreads();
  const bool b_fast_dst = p.db <= p.da;
  for (int k = t; k < n; k += 256) {
    int al, bl, tp;
    if (p.dt == 1) {
      tp = k % p.T;
      const int r = k / p.T;
      if (b_fast_dst) { bl = r % WS_T; al = r / WS_T; } else { al = r % WS_T; bl = r / WS_T; }
    } else {
      const int r = k % (WS_T * WS_T);
      tp = k / (WS_T * WS_T);
      if (b_fast_dst) { bl = r % WS_T; al = r / WS_T; } else { al = r % WS_T; bl = r / WS_T; }
    }
    const int a = a0 + al, b = b0 + bl;
    if (a < p.A && b < p.B) dst[o * p.dO + a * p.da + b * p.db + tp * p.dt] = tile[(al * WS_T + bl) * WR_TAPS + tp];
  }
}

}  // namespace vfd

using namespace vfd;

extern "C" {

int vfd_weight_fragments(int mode, const float* w, float* dst, int O, int C, int C1, int Z, int Cv, int D,
                         void* stream) {
  VFD_REQUIRE(w && dst && O > 0 && O % 4 == 0, "weight_fragments: bad arguments");
  WrArgs a{mode, O, C, C1, Z, Cv, D, 0, 0, 0};
  long long nrow = 0;
  if (mode == 0) {
    VFD_REQUIRE(C > 0 && (C1 <= 0 || (Z > 0 && C1 * Z == C)), "weight_fragments: C = %d vs C1 * Z", C);
    a.cpad = (C + 15) / 16 * 16;
    a.refperm = C1 > 0 ? 1 : 0;
    nrow = (long long)(a.cpad / 4) * O * 4;
  } else if (mode == 1) {
    VFD_REQUIRE(Cv > 0 && Cv % 4 == 0 && D > 0, "weight_fragments: Cv %% 4, D");
    nrow = (long long)D * (Cv / 4) * O * 4;
  } else if (mode == 2) {
    VFD_REQUIRE(Cv > 0 && D > 0, "weight_fragments: Cv, D");
    a.npad = (Cv * D + 255) / 256 * 256;
    nrow = (long long)(O / 4) * a.npad * 4;
  } else {
    set_error("weight_fragments: mode %d", mode);
    return VFD_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  if (mode == 1 && O % 16 == 0) {
    wfrag1_k<<<dim3((unsigned)(O / 16), (unsigned)(Cv / 4), (unsigned)((D + WT_DT - 1) / WT_DT)), 256, 0, s>>>(w, dst, O, Cv, D);
    return fail_launch("weight_fragments");
  }
  if (mode == 2 && Cv % 16 == 0) {
    wfrag2_k<<<dim3((unsigned)(O / 4), (unsigned)(Cv / 16), (unsigned)((D + WT_DT - 1) / WT_DT)), 256, 0, s>>>(w, dst, O, Cv, D,
                                                                                                        a.npad);
    if (a.npad > Cv * D) {
      const long long n = (long long)WR_TAPS * (O / 4) * (a.npad - Cv * D) * 4;
      wfrag2_pad_k<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(dst, O / 4, Cv * D, a.npad);
    }
    return fail_launch("weight_fragments");
  }
  if (mode == 0 && a.refperm && C1 % 4 == 0 && C % 16 == 0 && Z <= 40) {
    const size_t lds = (size_t)8 * 4 * Z * WR_TAPS * 4;
    wfrag0z_k<<<dim3((unsigned)((O + 7) / 8), (unsigned)(C1 / 4)), 256, lds, s>>>(w, dst, O, C1, Z);
    return fail_launch("weight_fragments");
  }
  weight_frag_k<<<(unsigned)((nrow + 255) / 256), 256, 0, s>>>(a, w, dst, nrow);
  return fail_launch("weight_fragments");
}

// bf16 fragment copies of the MFMA convolutions' weights (mode 3: K3C forward, projconv.hip
// pcvb_main_k); dst holds bf16 elements
int vfd_weight_fragments_bf16(int mode, const float* w, void* dst, int O, int C, int C1, int Z, int Cv, int D,
                              void* stream) {
  (void)C; (void)C1; (void)Z;
  VFD_REQUIRE(w && dst && O > 0, "weight_fragments_bf16: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  if (mode == 3) {
    VFD_REQUIRE(O % 32 == 0 && Cv > 0 && Cv % 16 == 0 && D > 0, "weight_fragments_bf16: mode 3 needs O %% 32, Cv %% 16");
    wfrag3_k<<<dim3((unsigned)(O / 32), (unsigned)(Cv / 16), (unsigned)((D + WT_D3 - 1) / WT_D3)), 256, 0, s>>>(
        w, (wbf16x8*)dst, O, Cv, D);
    return fail_launch("weight_fragments_bf16");
  }
  if (mode == 4) {          // w = the fp32 mode-0 fragment copy [9][ceil16(C)/4][O][2][2]
    VFD_REQUIRE(O % 32 == 0 && C > 0, "weight_fragments_bf16: mode 4 needs O %% 32");
    const int cq4 = (C + 15) / 16 * 4, nq16 = (C + 31) / 32 * 2;
    const long long n = (long long)WR_TAPS * nq16 * (O / 32) * 64;
    wfrag4_k<<<(unsigned)((n + 255) / 256), 256, 0, s>>>((const float4*)w, (wbf16x8*)dst, O, cq4, nq16);
    return fail_launch("weight_fragments_bf16");
  }
  if (mode == 5) {          // w = the fp32 mode-2 copy [9][O/4][npad][2][2] (K3C data gradient)
    VFD_REQUIRE(O % 16 == 0 && Cv > 0 && D > 0, "weight_fragments_bf16: mode 5 needs O %% 16");
    const int npad = (Cv * D + 255) / 256 * 256;
    const long long n = (long long)WR_TAPS * (O / 16) * (npad / 32) * 64;
    wfrag5_k<<<(unsigned)((n + 255) / 256), 256, 0, s>>>((const float4*)w, (wbf16x8*)dst, O / 4, npad);
    return fail_launch("weight_fragments_bf16");
  }
  set_error("weight_fragments_bf16: mode %d", mode);
  return VFD_EINVAL;
}

int vfd_weight_permute(const float* w, float* dst, int O, int A, int B, int T, const long long* src_strides,
                       const long long* dst_strides, void* stream) {
  VFD_REQUIRE(w && dst && src_strides && dst_strides && O > 0 && O < 65536 && A > 0 && B > 0 && T > 0 && T <= WR_TAPS,
              "weight_permute: bad arguments (taps <= %d)", WR_TAPS);
  WpArgs p;
  p.so = src_strides[0]; p.sa = src_strides[1]; p.sb = src_strides[2]; p.st = src_strides[3];
  p.dO = dst_strides[0]; p.da = dst_strides[1]; p.db = dst_strides[2]; p.dt = dst_strides[3];
  p.O = O; p.A = A; p.B = B; p.T = T;
  const int ta = (A + WS_T - 1) / WS_T;
  p.tiles_b = (B + WS_T - 1) / WS_T;
  hipStream_t s = (hipStream_t)stream;
  weight_permute_k<<<dim3((unsigned)(ta * p.tiles_b), (unsigned)O), 256, 0, s>>>(p, w, dst);
  return fail_launch("weight_permute");
}

int vfd_weight_swap(const float* w, float* dst, int O, int A, int B, int taps, void* stream) {
  const long long T = taps;
  const long long ss[4] = {(long long)A * B * T, B * T, T, 1};
  const long long ds[4] = {(long long)A * B * T, T, (long long)A * T, 1};
  return vfd_weight_permute(w, dst, O, A, B, taps, ss, ds, stream);
}

}  // extern "C"
