// Fused training-mode BatchNorm (+ residual) (+ ReLU) for the ResNet encoders of the fused depth /
// pose nets (network/fusion_depthnet.py:24-36, fusion_posenet.py:22-35: torchvision BasicBlock /
// Bottleneck + stem; under DDP their BN layers are SyncBatchNorm, models/vfdepth.py:68).
//
//   y = relu( (x - mean_c) * invstd_c * gamma_c + beta_c  [+ r] )        x, r, y: NCHW fp32
//
// MIOpen's BN kernel, the residual add and the ReLU are three HBM passes + launches per layer here
// (plus three more for their backward); these kernels do one statistics pass and one apply pass
// each way.  Statistics accumulate in fp64 (as the reference's CPU batch norm does), per
// (channel, split) partials summed in a fixed order: deterministic.  For SyncBatchNorm the host
// all-reduces the per-channel sums between the two passes (vfd_bn_sum): one collective per
// direction, the element count riding along as an extra row (no host synchronisation).
//
// Work split: a channel's N*HW elements (N images of HW contiguous floats) are cut into S
// equal float4-aligned ranges; block (split, channel) of every kernel owns one range.
//
// Groups (d.groups = G > 1): the tensors hold G consecutive batches of N images, each normalised
// with its OWN statistics — what G separate train-mode calls of the layer compute (the pose net's
// two frame-pair calls of a step run as one batch this way, fusion_posenet.py:42-72 /
// models/geometry/pose.py:33-42).  Block z = group; partials [G][C][S][2], reduced sums
// [G][C+1][2], mean / invstd [G][C]; the running statistics are updated G times in group order and
// num_batches_tracked grows by G (as after G calls); d gamma / d beta are the groups' values summed
// in fp32 in group order (autograd's accumulation over the calls).
#include "vfd_common.h"

namespace vfd {

constexpr int BN_THREADS = 256;

struct BnRange {
  unsigned lo, hi;      // element range [lo, hi) of the channel's N*HW (< 2^31, host-checked) elements
};

__device__ __forceinline__ BnRange bn_range(const vfd_bn_desc& d, int split) {
  const unsigned total = (unsigned)d.N * (unsigned)d.HW;
  const unsigned chunk = ((total + d.S - 1) / d.S + 3) & ~3u;
  BnRange r;
  r.lo = chunk * split;
  r.hi = r.lo + chunk < total ? r.lo + chunk : total;
  return r;
}

// element e of channel c -> offset in the NCHW tensor (32-bit division: the 64-bit one is a long
// software sequence per element)
__device__ __forceinline__ size_t bn_off(const vfd_bn_desc& d, int c, unsigned e) {
  const unsigned n = e / (unsigned)d.HW;
  return ((size_t)n * d.C + c) * d.HW + (e - n * (unsigned)d.HW);
}

__device__ __forceinline__ int bn_groups(const vfd_bn_desc& d) { return d.groups > 1 ? d.groups : 1; }
// elements of one group (N images)
__device__ __forceinline__ size_t bn_gsz(const vfd_bn_desc& d) { return (size_t)d.N * d.C * d.HW; }

// the running-statistics update of nn.BatchNorm2d.train() from one group's mean / biased variance
__device__ __forceinline__ void bn_running(const vfd_bn_desc& d, int c, double count, double mean_d, double var_d,
                                           float* __restrict__ run_mean, float* __restrict__ run_var) {
  const double unbiased = count > 1.0 ? var_d * count / (count - 1.0) : var_d;
  run_mean[c] = (float)((1.0 - d.momentum) * run_mean[c] + d.momentum * mean_d);
  run_var[c] = (float)((1.0 - d.momentum) * run_var[c] + d.momentum * unbiased);
}

__device__ __forceinline__ double block_sum(double v, double* sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wv] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < BN_THREADS / 64; ++i) s += sh[i];
  return s;
}

// Visit every element of a range: f(offset_of_float4, 4 values) with float4 loads when HW % 4 == 0.
template <typename F>
__device__ __forceinline__ void bn_visit(const vfd_bn_desc& d, int c, BnRange r, size_t gb, F&& f) {
  if ((d.HW & 3) == 0) {
#pragma unroll 2
    for (unsigned e = r.lo + 4 * threadIdx.x; e < r.hi; e += 4 * BN_THREADS) f(gb + bn_off(d, c, e), 4);
  } else {
    for (unsigned e = r.lo + threadIdx.x; e < r.hi; e += BN_THREADS) f(gb + bn_off(d, c, e), 1);
  }
}

// ReLU mask in the backward: from the forward output y (d.relu == 1) or from the forward's byte
// mask (d.relu == 2: `y` then points at N*C*HW bytes, 1 = positive output) — a quarter of the bytes
template <typename T>
__device__ __forceinline__ void relu_mask4(const vfd_bn_desc& d, const T* __restrict__ y, size_t o, float4& gv) {
  if (d.relu == 2) {
    const uchar4 m = *reinterpret_cast<const uchar4*>(reinterpret_cast<const unsigned char*>(y) + o);
    gv.x = m.x ? gv.x : 0.f;
    gv.y = m.y ? gv.y : 0.f;
    gv.z = m.z ? gv.z : 0.f;
    gv.w = m.w ? gv.w : 0.f;
  } else {
    const float4 yv = ld4(y + o);
    gv.x = yv.x > 0.f ? gv.x : 0.f;
    gv.y = yv.y > 0.f ? gv.y : 0.f;
    gv.z = yv.z > 0.f ? gv.z : 0.f;
    gv.w = yv.w > 0.f ? gv.w : 0.f;
  }
}

// the incoming gradient at element offset o (4 or 1 elements): g, plus the next block's identity-
// branch gradient g2 (masked by its ReLU byte mask m2) when d.g2 is set — summed in fp32 and
// rounded once to the activation type, exactly autograd's add of the two tensors
__device__ __forceinline__ float bn_rnd(float v, const float*) { return v; }
__device__ __forceinline__ float bn_rnd(float v, const __bf16*) { return (float)(__bf16)v; }

template <typename T>
__device__ __forceinline__ float4 bn_g4(const vfd_bn_desc& d, const T* __restrict__ g, size_t o) {
  float4 gv = ld4(g + o);
  if (d.g2) {
    float4 h = ld4(reinterpret_cast<const T*>(d.g2) + o);
    if (d.m2) {
      const uchar4 m = *reinterpret_cast<const uchar4*>(d.m2 + o);
      h.x = m.x ? h.x : 0.f;
      h.y = m.y ? h.y : 0.f;
      h.z = m.z ? h.z : 0.f;
      h.w = m.w ? h.w : 0.f;
    }
    gv.x = bn_rnd(gv.x + h.x, g);
    gv.y = bn_rnd(gv.y + h.y, g);
    gv.z = bn_rnd(gv.z + h.z, g);
    gv.w = bn_rnd(gv.w + h.w, g);
  }
  return gv;
}

template <typename T>
__device__ __forceinline__ float bn_g1(const vfd_bn_desc& d, const T* __restrict__ g, size_t o) {
  float gv = ld1(g + o);
  if (d.g2 && (!d.m2 || d.m2[o])) gv = bn_rnd(gv + ld1(reinterpret_cast<const T*>(d.g2) + o), g);
  return gv;
}

template <typename T>
__device__ __forceinline__ bool relu_on(const vfd_bn_desc& d, const T* __restrict__ y, size_t o) {
  return d.relu == 2 ? reinterpret_cast<const unsigned char*>(y)[o] != 0 : ld1(y + o) > 0.f;
}

// partial[(c*S + split)*2 + {0,1}] = sum x, sum x^2 over the range
template <typename T>
__global__ __launch_bounds__(BN_THREADS) void bn_stats_k(vfd_bn_desc d, const T* __restrict__ x,
                                                         double* __restrict__ partial) {
  __shared__ double sh[BN_THREADS / 64];
  const int c = blockIdx.y, split = blockIdx.x, grp = blockIdx.z;
  double s1 = 0.0, s2 = 0.0;
  bn_visit(d, c, bn_range(d, split), grp * bn_gsz(d), [&](size_t o, int n) {
    if (n == 4) {
      const float4 v = ld4(x + o);
      const double a = v.x, b = v.y, e = v.z, f = v.w;
      s1 += (a + b) + (e + f);
      s2 += (a * a + b * b) + (e * e + f * f);
    } else {
      const double a = ld1(x + o);
      s1 += a;
      s2 += a * a;
    }
  });
  s1 = block_sum(s1, sh);
  s2 = block_sum(s2, sh);
  if (threadIdx.x == 0) {
    partial[(((size_t)grp * d.C + c) * d.S + split) * 2] = s1;
    partial[(((size_t)grp * d.C + c) * d.S + split) * 2 + 1] = s2;
  }
}

// sums[c*2 + k] = sum over splits of partial (fixed order); one thread per channel.  SyncBatchNorm:
// thread C writes the local element count as row C (count > 0), so ONE all-reduce of the [C+1][2]
// buffer gives the global sums and the global count together (no host round trip for the count);
// dgamma / dbeta (backward, nullable) take this rank's LOCAL sums, as torch's SyncBatchNorm
// returns local parameter gradients that DDP then averages.
__global__ void bn_sum_k(vfd_bn_desc d, const double* __restrict__ partial, double count, double* __restrict__ sums,
                         const float* __restrict__ invstd, float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int G = bn_groups(d);
  const size_t sst = (size_t)(d.C + 1) * 2;          // one group's reduced sums
  if (c == d.C && count > 0.0) {
    for (int k = 0; k < G; ++k) {
      sums[k * sst + c * 2] = count;
      sums[k * sst + c * 2 + 1] = 0.0;
    }
  }
  if (c >= d.C) return;
  float dg = 0.f, db = 0.f;
  for (int k = 0; k < G; ++k) {
    const double* pk = partial + (size_t)k * d.C * d.S * 2;
    double a = 0.0, b = 0.0;
    for (int s = 0; s < d.S; ++s) {
      a += pk[((size_t)c * d.S + s) * 2];
      b += pk[((size_t)c * d.S + s) * 2 + 1];
    }
    sums[k * sst + c * 2] = a;
    sums[k * sst + c * 2 + 1] = b;
    if (dgamma) dg += (float)(b * invstd[(size_t)k * d.C + c]);
    if (dbeta) db += (float)a;
  }
  if (dgamma) dgamma[c] = dg;
  if (dbeta) dbeta[c] = db;
}

// per-channel sums of the block's channel: from the S partials, or (ns == 1) already reduced
// channel c's sums from its ns partials, by the whole block: thread i loads partial i (ns <= a few
// hundred), then a fixed-order block reduction — one round of loads instead of a serial chain of
// ns dependent ones in every thread (which dominated the apply kernels of the small layers)
__device__ __forceinline__ void bn_channel_sums(const double* __restrict__ part, int ns, int c, double* a,
                                                double* b) {
  __shared__ double sh[BN_THREADS / 64];
  double s1 = 0.0, s2 = 0.0;
  for (int s = threadIdx.x; s < ns; s += BN_THREADS) {
    s1 += part[((size_t)c * ns + s) * 2];
    s2 += part[((size_t)c * ns + s) * 2 + 1];
  }
  *a = block_sum(s1, sh);
  *b = block_sum(s2, sh);
}

// y = relu((x - mean) * invstd * gamma + beta [+ r]); block (0, c) also stores mean / invstd and
// updates the running statistics (momentum, unbiased variance), as nn.BatchNorm2d.train() does.
template <typename T>
__global__ __launch_bounds__(BN_THREADS) void bn_apply_k(vfd_bn_desc d, const T* __restrict__ x,
                                                         const T* __restrict__ r, const double* __restrict__ sums,
                                                         int ns, double count, const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, T* __restrict__ y,
                                                         float* __restrict__ mean_out, float* __restrict__ invstd_out,
                                                         float* __restrict__ run_mean, float* __restrict__ run_var,
                                                         long long* __restrict__ nbt, unsigned char* __restrict__ mk) {
  const int c = blockIdx.y, split = blockIdx.x, grp = blockIdx.z, G = bn_groups(d);
  if (nbt && c == 0 && split == 0 && grp == 0 && threadIdx.x == 0) nbt[0] += G;   // num_batches_tracked
  const size_t sst = ns == 1 ? (size_t)(d.C + 1) * 2 : (size_t)d.C * d.S * 2;   // one group's sums
  const double cnt = count > 0.0 ? count : sums[grp * sst + 2 * d.C];   // all-reduced count row (ns == 1)
  double s1, s2;
  bn_channel_sums(sums + grp * sst, ns, c, &s1, &s2);
  const double mean_d = s1 / cnt;
  double var_d = s2 / cnt - mean_d * mean_d;
  var_d = var_d > 0.0 ? var_d : 0.0;
  const float mean = (float)mean_d;
  const float invstd = (float)(1.0 / sqrt(var_d + (double)d.eps));
  if (split == 0 && threadIdx.x == 0) {
    mean_out[(size_t)grp * d.C + c] = mean;
    invstd_out[(size_t)grp * d.C + c] = invstd;
  }
  if (run_mean && split == 0 && grp == 0) {      // block-uniform: the groups' updates in order
    for (int k = 0; k < G; ++k) {
      double a = s1, b = s2, ck = cnt;
      if (k > 0) {
        ck = count > 0.0 ? count : sums[k * sst + 2 * d.C];
        bn_channel_sums(sums + k * sst, ns, c, &a, &b);
      }
      const double mk_d = a / ck;
      double vk = b / ck - mk_d * mk_d;
      vk = vk > 0.0 ? vk : 0.0;
      if (threadIdx.x == 0) bn_running(d, c, ck, mk_d, vk, run_mean, run_var);
    }
  }
  const float sc = invstd * gamma[c];
  const float sh = beta[c] - mean * sc;
  const bool relu = d.relu != 0;
  bn_visit(d, c, bn_range(d, split), grp * bn_gsz(d), [&](size_t o, int n) {
    if (n == 4) {
      float4 v = ld4(x + o);
      v.x = v.x * sc + sh;
      v.y = v.y * sc + sh;
      v.z = v.z * sc + sh;
      v.w = v.w * sc + sh;
      if (r) {
        const float4 q = ld4(r + o);
        v.x += q.x;
        v.y += q.y;
        v.z += q.z;
        v.w += q.w;
      }
      if (relu) {
        v.x = fmaxf(v.x, 0.f);
        v.y = fmaxf(v.y, 0.f);
        v.z = fmaxf(v.z, 0.f);
        v.w = fmaxf(v.w, 0.f);
      }
      st4(y + o, v);
      if (mk) *reinterpret_cast<uchar4*>(mk + o) = make_uchar4(v.x > 0.f, v.y > 0.f, v.z > 0.f, v.w > 0.f);
    } else {
      float v = ld1(x + o) * sc + sh;
      if (r) v += ld1(r + o);
      if (relu) v = fmaxf(v, 0.f);
      st1(y + o, v);
      if (mk) mk[o] = v > 0.f;
    }
  });
}

// backward statistics: sum g', sum g' * (x - mean), g' = g * [y > 0] (relu) or g
template <typename T>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_stats_k(vfd_bn_desc d, const T* __restrict__ g,
                                                             const T* __restrict__ y, const T* __restrict__ x,
                                                             const float* __restrict__ mean_in,
                                                             double* __restrict__ partial) {
  __shared__ double sh[BN_THREADS / 64];
  const int c = blockIdx.y, split = blockIdx.x, grp = blockIdx.z;
  const float mean = mean_in[(size_t)grp * d.C + c];
  const bool relu = d.relu != 0;
  double s1 = 0.0, s2 = 0.0;
  bn_visit(d, c, bn_range(d, split), grp * bn_gsz(d), [&](size_t o, int n) {
    if (n == 4) {
      float4 gv = bn_g4(d, g, o);
      const float4 xv = ld4(x + o);
      if (relu) relu_mask4(d, y, o, gv);
      s1 += ((double)gv.x + (double)gv.y) + ((double)gv.z + (double)gv.w);
      s2 += ((double)gv.x * (double)(xv.x - mean) + (double)gv.y * (double)(xv.y - mean)) +
            ((double)gv.z * (double)(xv.z - mean) + (double)gv.w * (double)(xv.w - mean));
    } else {
      float gv = bn_g1(d, g, o);
      if (relu && !relu_on(d, y, o)) gv = 0.f;
      s1 += gv;
      s2 += (double)gv * (double)(ld1(x + o) - mean);
    }
  });
  s1 = block_sum(s1, sh);
  s2 = block_sum(s2, sh);
  if (threadIdx.x == 0) {
    partial[(((size_t)grp * d.C + c) * d.S + split) * 2] = s1;
    partial[(((size_t)grp * d.C + c) * d.S + split) * 2 + 1] = s2;
  }
}

// dx = gamma * invstd * (g' - sum g'/n - (x - mean) * invstd^2 * sum g'(x - mean) / n); dr = g';
// block (0, c) stores d gamma = invstd * sum g'(x - mean), d beta = sum g'
template <typename T>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_apply_k(vfd_bn_desc d, const T* __restrict__ g,
                                                             const T* __restrict__ y, const T* __restrict__ x,
                                                             const double* __restrict__ sums, int ns, double count,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ mean_in,
                                                             const float* __restrict__ invstd_in,
                                                             T* __restrict__ dx, T* __restrict__ dr,
                                                             float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int c = blockIdx.y, split = blockIdx.x, grp = blockIdx.z, G = bn_groups(d);
  const size_t sst = ns == 1 ? (size_t)(d.C + 1) * 2 : (size_t)d.C * d.S * 2;   // one group's sums
  const double cnt = count > 0.0 ? count : sums[grp * sst + 2 * d.C];   // all-reduced count row (ns == 1)
  double sg, sgx;
  bn_channel_sums(sums + grp * sst, ns, c, &sg, &sgx);
  const float mean = mean_in[(size_t)grp * d.C + c], invstd = invstd_in[(size_t)grp * d.C + c];
  if (split == 0 && grp == 0 && (dgamma || dbeta)) {   // block-uniform: the groups' values, fp32, in order
    float dg = 0.f, db = 0.f;
    for (int k = 0; k < G; ++k) {
      double a = sg, b = sgx;
      if (k > 0) bn_channel_sums(sums + k * sst, ns, c, &a, &b);
      dg += (float)(b * invstd_in[(size_t)k * d.C + c]);
      db += (float)a;
    }
    if (threadIdx.x == 0) {
      if (dgamma) dgamma[c] = dg;
      if (dbeta) dbeta[c] = db;
    }
  }
  const float k = gamma[c] * invstd;
  const float mg = (float)(sg / cnt);
  const float mx = (float)(sgx / cnt) * invstd * invstd;
  const bool relu = d.relu != 0;
  bn_visit(d, c, bn_range(d, split), grp * bn_gsz(d), [&](size_t o, int n) {
    if (n == 4) {
      float4 gv = bn_g4(d, g, o);
      const float4 xv = ld4(x + o);
      if (relu) relu_mask4(d, y, o, gv);
      if (dr) st4(dr + o, gv);
      if (dx) {
        float4 o4;
        o4.x = k * (gv.x - mg - (xv.x - mean) * mx);
        o4.y = k * (gv.y - mg - (xv.y - mean) * mx);
        o4.z = k * (gv.z - mg - (xv.z - mean) * mx);
        o4.w = k * (gv.w - mg - (xv.w - mean) * mx);
        st4(dx + o, o4);
      }
    } else {
      float gv = bn_g1(d, g, o);
      if (relu && !relu_on(d, y, o)) gv = 0.f;
      if (dr) st1(dr + o, gv);
      if (dx) st1(dx + o, k * (gv - mg - (ld1(x + o) - mean) * mx));
    }
  });
}


// ---- one-launch variants for channels of at most BN1_MAX elements (the 1/16 - 1/32 ResNet layers,
// local statistics only): one workgroup per channel computes the statistics and then applies them
// (the second sweep re-reads the channel from L2), so a layer is one launch each way instead of
// two, and no partials round-trip through memory.  Fixed summation order: deterministic.
constexpr int BN1_THREADS = 512;
// (channels-last maps take the 3-launch split path: a one-launch NHWC form, a block per 8 channels,
// measured slower — config 3 BN 4.50 vs 3.86 ms/step with C / 8 blocks per layer — and was retired
// in round 6)
constexpr unsigned BN1_MAX = 8192;   // layer2 (23040 / channel) keeps the split path: its 128 channels alone would leave half the CUs idle

__device__ __forceinline__ double block_sum1(double v, double* sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wv] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < BN1_THREADS / 64; ++i) s += sh[i];
  return s;
}

template <typename F>
__device__ __forceinline__ void bn1_visit(const vfd_bn_desc& d, int c, size_t gb, F&& f) {
  const unsigned total = (unsigned)d.N * (unsigned)d.HW;
  if ((d.HW & 3) == 0) {
    for (unsigned e = 4 * threadIdx.x; e < total; e += 4 * BN1_THREADS) f(gb + bn_off(d, c, e), 4);
  } else {
    for (unsigned e = threadIdx.x; e < total; e += BN1_THREADS) f(gb + bn_off(d, c, e), 1);
  }
}

template <typename T>
__global__ __launch_bounds__(BN1_THREADS) void bn1_fwd_k(vfd_bn_desc d, const T* __restrict__ x,
                                                         const T* __restrict__ r, const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, T* __restrict__ y,
                                                         float* __restrict__ mean_out, float* __restrict__ invstd_out,
                                                         float* __restrict__ run_mean, float* __restrict__ run_var,
                                                         long long* __restrict__ nbt, unsigned char* __restrict__ mk) {
  __shared__ double sh[BN1_THREADS / 64];
  const int c = blockIdx.x, G = bn_groups(d);
  if (nbt && c == 0 && threadIdx.x == 0) nbt[0] += G;
  for (int grp = 0; grp < G; ++grp) {          // the groups in order (running statistics)
  const size_t gb = grp * bn_gsz(d);
  double s1 = 0.0, s2 = 0.0;
  bn1_visit(d, c, gb, [&](size_t o, int n) {
    if (n == 4) {
      const float4 v = ld4(x + o);
      const double a = v.x, b = v.y, e = v.z, f = v.w;
      s1 += (a + b) + (e + f);
      s2 += (a * a + b * b) + (e * e + f * f);
    } else {
      const double a = ld1(x + o);
      s1 += a;
      s2 += a * a;
    }
  });
  s1 = block_sum1(s1, sh);
  s2 = block_sum1(s2, sh);
  const double count = (double)d.N * d.HW;
  const double mean_d = s1 / count;
  double var_d = s2 / count - mean_d * mean_d;
  var_d = var_d > 0.0 ? var_d : 0.0;
  const float mean = (float)mean_d;
  const float invstd = (float)(1.0 / sqrt(var_d + (double)d.eps));
  if (threadIdx.x == 0) {
    mean_out[(size_t)grp * d.C + c] = mean;
    invstd_out[(size_t)grp * d.C + c] = invstd;
    if (run_mean) bn_running(d, c, count, mean_d, var_d, run_mean, run_var);
  }
  const float sc = invstd * gamma[c];
  const float shf = beta[c] - mean * sc;
  const bool relu = d.relu != 0;
  bn1_visit(d, c, gb, [&](size_t o, int n) {
    if (n == 4) {
      float4 v = ld4(x + o);
      v.x = v.x * sc + shf;
      v.y = v.y * sc + shf;
      v.z = v.z * sc + shf;
      v.w = v.w * sc + shf;
      if (r) {
        const float4 q = ld4(r + o);
        v.x += q.x;
        v.y += q.y;
        v.z += q.z;
        v.w += q.w;
      }
      if (relu) {
        v.x = fmaxf(v.x, 0.f);
        v.y = fmaxf(v.y, 0.f);
        v.z = fmaxf(v.z, 0.f);
        v.w = fmaxf(v.w, 0.f);
      }
      st4(y + o, v);
      if (mk) *reinterpret_cast<uchar4*>(mk + o) = make_uchar4(v.x > 0.f, v.y > 0.f, v.z > 0.f, v.w > 0.f);
    } else {
      float v = ld1(x + o) * sc + shf;
      if (r) v += ld1(r + o);
      if (relu) v = fmaxf(v, 0.f);
      st1(y + o, v);
      if (mk) mk[o] = v > 0.f;
    }
  });
  }
}

template <typename T>
__global__ __launch_bounds__(BN1_THREADS) void bn1_bwd_k(vfd_bn_desc d, const T* __restrict__ g,
                                                         const T* __restrict__ y, const T* __restrict__ x,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ mean_in,
                                                         const float* __restrict__ invstd_in, T* __restrict__ dx,
                                                         T* __restrict__ dr, float* __restrict__ dgamma,
                                                         float* __restrict__ dbeta) {
  __shared__ double sh[BN1_THREADS / 64];
  const int c = blockIdx.x, G = bn_groups(d);
  const bool relu = d.relu != 0;
  float dg = 0.f, db = 0.f;
  for (int grp = 0; grp < G; ++grp) {
  const size_t gb = grp * bn_gsz(d);
  const float mean = mean_in[(size_t)grp * d.C + c], invstd = invstd_in[(size_t)grp * d.C + c];
  double s1 = 0.0, s2 = 0.0;
  bn1_visit(d, c, gb, [&](size_t o, int n) {
    if (n == 4) {
      float4 gv = bn_g4(d, g, o);
      const float4 xv = ld4(x + o);
      if (relu) relu_mask4(d, y, o, gv);
      s1 += ((double)gv.x + (double)gv.y) + ((double)gv.z + (double)gv.w);
      s2 += ((double)gv.x * (double)(xv.x - mean) + (double)gv.y * (double)(xv.y - mean)) +
            ((double)gv.z * (double)(xv.z - mean) + (double)gv.w * (double)(xv.w - mean));
    } else {
      float gv = bn_g1(d, g, o);
      if (relu && !relu_on(d, y, o)) gv = 0.f;
      s1 += gv;
      s2 += (double)gv * (double)(ld1(x + o) - mean);
    }
  });
  const double sg = block_sum1(s1, sh), sgx = block_sum1(s2, sh);
  dg += (float)(sgx * invstd);
  db += (float)sg;
  const double count = (double)d.N * d.HW;
  const float k = gamma[c] * invstd;
  const float mg = (float)(sg / count);
  const float mx = (float)(sgx / count) * invstd * invstd;
  bn1_visit(d, c, gb, [&](size_t o, int n) {
    if (n == 4) {
      float4 gv = bn_g4(d, g, o);
      const float4 xv = ld4(x + o);
      if (relu) relu_mask4(d, y, o, gv);
      if (dr) st4(dr + o, gv);
      if (dx) {
        float4 o4;
        o4.x = k * (gv.x - mg - (xv.x - mean) * mx);
        o4.y = k * (gv.y - mg - (xv.y - mean) * mx);
        o4.z = k * (gv.z - mg - (xv.z - mean) * mx);
        o4.w = k * (gv.w - mg - (xv.w - mean) * mx);
        st4(dx + o, o4);
      }
    } else {
      float gv = bn_g1(d, g, o);
      if (relu && !relu_on(d, y, o)) gv = 0.f;
      if (dr) st1(dr + o, gv);
      if (dx) st1(dx + o, k * (gv - mg - (ld1(x + o) - mean) * mx));
    }
  });
  }
  if (threadIdx.x == 0) {
    if (dgamma) dgamma[c] = dg;
    if (dbeta) dbeta[c] = db;
  }
}

// ---- channels-last (d.nhwc = 1): config 3's bf16 encoders keep their maps NHWC so MIOpen's
// convolutions run without their NCHW <-> NHWC transposes.  x is [R = N*HW rows][C]; a row's C
// channels are contiguous, so a channel's statistics cannot be one block's contiguous range:
// block `split` of the statistics kernels owns rows [split*chunk, ...) of ALL channels, thread t
// the channel quad(s) q = t % QW (+ 256 j) of every RP-th row, and the per-(channel, split)
// partials keep the NCHW path's [C][S][2] layout (vfd_bn_sum reduces them in a fixed order).
// The apply passes read reduced sums (ns = 1): each block first turns them into per-channel
// coefficients in LDS, then streams float4s of [R][C] (quad = index mod C/4).
constexpr int NH_MAXC = 2048;        // ResNet-50's widest stage; C/4 a power of two

struct NhGeom {
  unsigned rows, chunk;   // R = N*HW, rows per split
  int Q, QW, QT, RP;      // quads per row, quads per thread-row group (<= 256), quads per thread, rows per sweep
};

__device__ __forceinline__ NhGeom nh_geom(const vfd_bn_desc& d) {
  NhGeom g;
  g.rows = (unsigned)d.N * (unsigned)d.HW;
  g.chunk = (g.rows + d.S - 1) / d.S;
  g.Q = d.C >> 2;
  g.QW = g.Q < BN_THREADS ? g.Q : BN_THREADS;
  g.QT = g.Q / g.QW;
  g.RP = BN_THREADS / g.QW;
  return g;
}

// per-thread channel accumulators (QT <= 2) -> per-(channel, split) partials, rows summed in order
__device__ __forceinline__ void nh_store_partials(const vfd_bn_desc& d, const NhGeom& g, double (&a)[2][4],
                                                  double (&b)[2][4], double* __restrict__ partial) {
  const int q0 = threadIdx.x % g.QW, rs = threadIdx.x / g.QW;
  if (g.RP == 1) {        // C >= 1024: every thread owns whole channels
    for (int j = 0; j < g.QT; ++j)
      for (int k = 0; k < 4; ++k) {
        const int c = 4 * (q0 + j * g.QW) + k;
        partial[((size_t)c * d.S + blockIdx.x) * 2] = a[j][k];
        partial[((size_t)c * d.S + blockIdx.x) * 2 + 1] = b[j][k];
      }
    return;
  }
  __shared__ double s1[4 * BN_THREADS];     // [RP][C], RP * C = 4 * BN_THREADS when C < 1024
  __shared__ double s2[4 * BN_THREADS];
  for (int j = 0; j < g.QT; ++j)
    for (int k = 0; k < 4; ++k) {
      const int slot = rs * d.C + 4 * (q0 + j * g.QW) + k;    // [RP][C]
      s1[slot] = a[j][k];
      s2[slot] = b[j][k];
    }
  __syncthreads();
  for (int c = threadIdx.x; c < d.C; c += BN_THREADS) {
    double u = 0.0, v = 0.0;
    for (int r = 0; r < g.RP; ++r) {
      u += s1[r * d.C + c];
      v += s2[r * d.C + c];
    }
    partial[((size_t)c * d.S + blockIdx.x) * 2] = u;
    partial[((size_t)c * d.S + blockIdx.x) * 2 + 1] = v;
  }
}

template <typename T>
__global__ __launch_bounds__(BN_THREADS) void bn_stats_nhwc_k(vfd_bn_desc d, const T* __restrict__ x,
                                                              double* __restrict__ partial) {
  const NhGeom g = nh_geom(d);
  const int q0 = threadIdx.x % g.QW, rs = threadIdx.x / g.QW, grp = blockIdx.y;
  const unsigned lo = blockIdx.x * g.chunk, hi = lo + g.chunk < g.rows ? lo + g.chunk : g.rows;
  const size_t gb = grp * bn_gsz(d);
  double a[2][4] = {}, b[2][4] = {};
  for (unsigned r = lo + rs; r < hi; r += g.RP)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j >= g.QT) break;
      const float4 v = ld4(x + gb + (size_t)r * d.C + 4 * (q0 + j * g.QW));
      a[j][0] += v.x; a[j][1] += v.y; a[j][2] += v.z; a[j][3] += v.w;
      b[j][0] += (double)v.x * v.x; b[j][1] += (double)v.y * v.y;
      b[j][2] += (double)v.z * v.z; b[j][3] += (double)v.w * v.w;
    }
  nh_store_partials(d, g, a, b, partial + (size_t)grp * d.C * d.S * 2);
}

template <typename T>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_stats_nhwc_k(vfd_bn_desc d, const T* __restrict__ gr,
                                                                  const T* __restrict__ y, const T* __restrict__ x,
                                                                  const float* __restrict__ mean_in,
                                                                  double* __restrict__ partial) {
  const NhGeom g = nh_geom(d);
  const int q0 = threadIdx.x % g.QW, rs = threadIdx.x / g.QW, grp = blockIdx.y;
  const unsigned lo = blockIdx.x * g.chunk, hi = lo + g.chunk < g.rows ? lo + g.chunk : g.rows;
  const size_t gb = grp * bn_gsz(d);
  float4 mu[2];
  for (int j = 0; j < g.QT; ++j)
    mu[j] = *reinterpret_cast<const float4*>(mean_in + (size_t)grp * d.C + 4 * (q0 + j * g.QW));
  const bool relu = d.relu != 0;
  double a[2][4] = {}, b[2][4] = {};
  for (unsigned r = lo + rs; r < hi; r += g.RP)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j >= g.QT) break;
      const size_t o = gb + (size_t)r * d.C + 4 * (q0 + j * g.QW);
      float4 gv = bn_g4(d, gr, o);
      const float4 xv = ld4(x + o);
      if (relu) relu_mask4(d, y, o, gv);
      a[j][0] += gv.x; a[j][1] += gv.y; a[j][2] += gv.z; a[j][3] += gv.w;
      b[j][0] += (double)gv.x * (double)(xv.x - mu[j].x);
      b[j][1] += (double)gv.y * (double)(xv.y - mu[j].y);
      b[j][2] += (double)gv.z * (double)(xv.z - mu[j].z);
      b[j][3] += (double)gv.w * (double)(xv.w - mu[j].w);
    }
  nh_store_partials(d, g, a, b, partial + (size_t)grp * d.C * d.S * 2);
}

// sums[c] from the S partials by one block per channel (the NHWC path has hundreds of splits: a
// serial chain per thread would dominate); block C writes the count row
__global__ __launch_bounds__(BN_THREADS) void bn_sum_blk_k(vfd_bn_desc d, const double* __restrict__ partial,
                                                           double count, double* __restrict__ sums,
                                                           const float* __restrict__ invstd,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int c = blockIdx.x, G = bn_groups(d);
  const size_t sst = (size_t)(d.C + 1) * 2;          // one group's reduced sums
  if (c == d.C) {
    if (count > 0.0 && threadIdx.x == 0)
      for (int k = 0; k < G; ++k) {
        sums[k * sst + c * 2] = count;
        sums[k * sst + c * 2 + 1] = 0.0;
      }
    return;
  }
  float dg = 0.f, db = 0.f;
  for (int k = 0; k < G; ++k) {
    double a, b;
    bn_channel_sums(partial + (size_t)k * d.C * d.S * 2, d.S, c, &a, &b);
    if (threadIdx.x == 0) {
      sums[k * sst + c * 2] = a;
      sums[k * sst + c * 2 + 1] = b;
      if (dgamma) dg += (float)(b * invstd[(size_t)k * d.C + c]);
      if (dbeta) db += (float)a;
    }
  }
  if (threadIdx.x == 0) {
    if (dgamma) dgamma[c] = dg;
    if (dbeta) dbeta[c] = db;
  }
}

template <typename T>
__global__ __launch_bounds__(BN_THREADS) void bn_apply_nhwc_k(vfd_bn_desc d, const T* __restrict__ x,
                                                              const T* __restrict__ r, const double* __restrict__ sums,
                                                              double count, const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, T* __restrict__ y,
                                                              float* __restrict__ mean_out,
                                                              float* __restrict__ invstd_out,
                                                              float* __restrict__ run_mean, float* __restrict__ run_var,
                                                              long long* __restrict__ nbt,
                                                              unsigned char* __restrict__ mk) {
  __shared__ float2 coef[NH_MAXC];
  const int grp = blockIdx.y, G = bn_groups(d);
  if (nbt && blockIdx.x == 0 && grp == 0 && threadIdx.x == 0) nbt[0] += G;
  const size_t sst = (size_t)(d.C + 1) * 2;          // one group's reduced sums
  const double* sg = sums + grp * sst;
  const double cnt = count > 0.0 ? count : sg[2 * d.C];
  for (int c = threadIdx.x; c < d.C; c += BN_THREADS) {     // the NCHW apply's per-channel arithmetic
    const double mean_d = sg[2 * c] / cnt;
    double var_d = sg[2 * c + 1] / cnt - mean_d * mean_d;
    var_d = var_d > 0.0 ? var_d : 0.0;
    const float mean = (float)mean_d;
    const float invstd = (float)(1.0 / sqrt(var_d + (double)d.eps));
    const float sc = invstd * gamma[c];
    coef[c] = make_float2(sc, beta[c] - mean * sc);
    if (blockIdx.x == 0) {
      mean_out[(size_t)grp * d.C + c] = mean;
      invstd_out[(size_t)grp * d.C + c] = invstd;
      if (run_mean && grp == 0)                  // the groups' updates in order
        for (int k = 0; k < G; ++k) {
          const double* sk = sums + k * sst;
          const double ck = count > 0.0 ? count : sk[2 * d.C];
          const double mk_d = sk[2 * c] / ck;
          double vk = sk[2 * c + 1] / ck - mk_d * mk_d;
          vk = vk > 0.0 ? vk : 0.0;
          bn_running(d, c, ck, mk_d, vk, run_mean, run_var);
        }
    }
  }
  __syncthreads();
  const unsigned qm = (unsigned)(d.C >> 2) - 1u;
  const unsigned total4 = (unsigned)d.N * (unsigned)d.HW * (unsigned)(d.C >> 2);
  const bool relu = d.relu != 0;
  const size_t gb = grp * bn_gsz(d);
  for (unsigned i = blockIdx.x * BN_THREADS + threadIdx.x; i < total4; i += gridDim.x * BN_THREADS) {
    const size_t o = gb + 4 * (size_t)i;
    const int c = 4 * (i & qm);
    float4 v = ld4(x + o);
    const float2 k0 = coef[c], k1 = coef[c + 1], k2 = coef[c + 2], k3 = coef[c + 3];
    v.x = v.x * k0.x + k0.y;
    v.y = v.y * k1.x + k1.y;
    v.z = v.z * k2.x + k2.y;
    v.w = v.w * k3.x + k3.y;
    if (r) {
      const float4 q = ld4(r + o);
      v.x += q.x;
      v.y += q.y;
      v.z += q.z;
      v.w += q.w;
    }
    if (relu) {
      v.x = fmaxf(v.x, 0.f);
      v.y = fmaxf(v.y, 0.f);
      v.z = fmaxf(v.z, 0.f);
      v.w = fmaxf(v.w, 0.f);
    }
    st4(y + o, v);
    if (mk) *reinterpret_cast<uchar4*>(mk + o) = make_uchar4(v.x > 0.f, v.y > 0.f, v.z > 0.f, v.w > 0.f);
  }
}

template <typename T>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_apply_nhwc_k(vfd_bn_desc d, const T* __restrict__ g,
                                                                  const T* __restrict__ y, const T* __restrict__ x,
                                                                  const double* __restrict__ sums, double count,
                                                                  const float* __restrict__ gamma,
                                                                  const float* __restrict__ mean_in,
                                                                  const float* __restrict__ invstd_in,
                                                                  T* __restrict__ dx, T* __restrict__ dr,
                                                                  float* __restrict__ dgamma,
                                                                  float* __restrict__ dbeta) {
  __shared__ float4 coef[NH_MAXC];     // k, mean g', mx, mean
  const int grp = blockIdx.y, G = bn_groups(d);
  const size_t sst = (size_t)(d.C + 1) * 2;          // one group's reduced sums
  const double cnt = count > 0.0 ? count : sums[grp * sst + 2 * d.C];
  for (int c = threadIdx.x; c < d.C; c += BN_THREADS) {
    const double sg = sums[grp * sst + 2 * c], sgx = sums[grp * sst + 2 * c + 1];
    const float mean = mean_in[(size_t)grp * d.C + c], invstd = invstd_in[(size_t)grp * d.C + c];
    if (blockIdx.x == 0 && grp == 0 && (dgamma || dbeta)) {   // the groups' values, fp32, in order
      float dg = 0.f, db = 0.f;
      for (int k = 0; k < G; ++k) {
        dg += (float)(sums[k * sst + 2 * c + 1] * invstd_in[(size_t)k * d.C + c]);
        db += (float)sums[k * sst + 2 * c];
      }
      if (dgamma) dgamma[c] = dg;
      if (dbeta) dbeta[c] = db;
    }
    coef[c] = make_float4(gamma[c] * invstd, (float)(sg / cnt), (float)(sgx / cnt) * invstd * invstd, mean);
  }
  __syncthreads();
  const unsigned qm = (unsigned)(d.C >> 2) - 1u;
  const unsigned total4 = (unsigned)d.N * (unsigned)d.HW * (unsigned)(d.C >> 2);
  const bool relu = d.relu != 0;
  const size_t gb = grp * bn_gsz(d);
  for (unsigned i = blockIdx.x * BN_THREADS + threadIdx.x; i < total4; i += gridDim.x * BN_THREADS) {
    const size_t o = gb + 4 * (size_t)i;
    const int c = 4 * (i & qm);
    float4 gv = bn_g4(d, g, o);
    if (relu) relu_mask4(d, y, o, gv);
    if (dr) st4(dr + o, gv);
    if (dx) {
      const float4 xv = ld4(x + o);
      const float4 k0 = coef[c], k1 = coef[c + 1], k2 = coef[c + 2], k3 = coef[c + 3];
      float4 o4;
      o4.x = k0.x * (gv.x - k0.y - (xv.x - k0.w) * k0.z);
      o4.y = k1.x * (gv.y - k1.y - (xv.y - k1.w) * k1.z);
      o4.z = k2.x * (gv.z - k2.y - (xv.z - k2.w) * k2.z);
      o4.w = k3.x * (gv.w - k3.y - (xv.w - k3.w) * k3.z);
      st4(dx + o, o4);
    }
  }
}

}  // namespace vfd

using namespace vfd;

// grid of the NHWC apply passes: ~4 float4 per thread, at most 4096 blocks
static int nh_apply_blocks(const vfd_bn_desc* d) {
  const long long total4 = (long long)d->N * d->HW * (d->C >> 2);
  long long b = (total4 + 4 * BN_THREADS - 1) / (4 * BN_THREADS);
  return (int)(b < 1 ? 1 : b > 4096 ? 4096 : b);
}

extern "C" {

int vfd_bn_splits(const vfd_bn_desc* d) {
  if (!d || d->N <= 0 || d->C <= 0 || d->HW <= 0) return 0;
  if (d->nhwc) {          // row splits over all channels: ~4k elements per block, at most 2048
    const long long rows = (long long)d->N * d->HW;
    long long s = (rows * d->C + 4095) / 4096;
    if (s > 2048) s = 2048;
    if (s > rows) s = rows;
    return (int)(s < 1 ? 1 : s);
  }
  // ~4096 blocks per pass, >= 2048 elements per block
  const long long total = (long long)d->N * d->HW;
  long long s = (4096 + d->C - 1) / d->C;
  const long long most = (total + 2047) / 2048;
  if (s > most) s = most;
  if (s < 1) s = 1;
  return (int)s;
}

static int bn_check(const vfd_bn_desc* d, const char* what) {
  VFD_REQUIRE(d && d->N > 0 && d->C > 0 && d->HW > 0 && d->S > 0 && d->S == vfd_bn_splits(d),
              "%s: bad descriptor (S must be vfd_bn_splits)", what);
  VFD_REQUIRE((long long)d->N * d->HW < (1LL << 31), "%s: more than 2^31 elements per channel", what);
  VFD_REQUIRE(d->groups >= 0 && d->groups <= 64, "%s: groups must be in [0, 64]", what);
  if (d->nhwc)
    VFD_REQUIRE(d->C % 4 == 0 && d->C <= NH_MAXC && ((d->C >> 2) & ((d->C >> 2) - 1)) == 0 &&
                    (long long)d->N * d->HW * d->C < (1LL << 31),
                "%s: channels-last needs C/4 a power of two, C <= %d and < 2^31 elements", what, NH_MAXC);
  return VFD_OK;
}

int vfd_bn_fwd_stats(const vfd_bn_desc* d, const void* x, double* partial, void* stream) {
  if (int e = bn_check(d, "bn_fwd_stats")) return e;
  VFD_REQUIRE(x && partial, "bn_fwd_stats: null argument");
  hipStream_t s = (hipStream_t)stream;
  const int G = d->groups > 1 ? d->groups : 1;
  ProfScope ps(K_BN_FWD, s);
  if (d->nhwc) {
    if (d->dtype == 1) bn_stats_nhwc_k<__bf16><<<dim3(d->S, G), BN_THREADS, 0, s>>>(*d, (const __bf16*)x, partial);
    else bn_stats_nhwc_k<float><<<dim3(d->S, G), BN_THREADS, 0, s>>>(*d, (const float*)x, partial);
    return fail_launch("bn_fwd_stats");
  }
  if (d->dtype == 1) bn_stats_k<__bf16><<<dim3(d->S, d->C, G), BN_THREADS, 0, s>>>(*d, (const __bf16*)x, partial);
  else bn_stats_k<float><<<dim3(d->S, d->C, G), BN_THREADS, 0, s>>>(*d, (const float*)x, partial);
  return fail_launch("bn_fwd_stats");
}

int vfd_bn_sum(const vfd_bn_desc* d, const double* partial, double count, double* sums, const float* invstd,
               float* dgamma, float* dbeta, void* stream) {
  if (int e = bn_check(d, "bn_sum")) return e;
  VFD_REQUIRE(partial && sums, "bn_sum: null argument");
  VFD_REQUIRE(invstd || (!dgamma && !dbeta), "bn_sum: dgamma / dbeta need invstd");
  hipStream_t s = (hipStream_t)stream;
  if (d->S > 64) {
    bn_sum_blk_k<<<d->C + 1, BN_THREADS, 0, s>>>(*d, partial, count, sums, invstd, dgamma, dbeta);
    return fail_launch("bn_sum");
  }
  bn_sum_k<<<(d->C + 1 + 255) / 256, 256, 0, s>>>(*d, partial, count, sums, invstd, dgamma, dbeta);
  return fail_launch("bn_sum");
}

int vfd_bn_fwd_apply(const vfd_bn_desc* d, const void* x, const void* residual, const double* sums, int ns,
                     double count, const float* gamma, const float* beta, void* y, float* mean, float* invstd,
                     float* running_mean, float* running_var, long long* num_batches_tracked,
                     unsigned char* relu_mask, void* stream) {
  if (int e = bn_check(d, "bn_fwd_apply")) return e;
  const int G = d->groups > 1 ? d->groups : 1;
  VFD_REQUIRE(x && sums && gamma && beta && y && mean && invstd && (ns == 1 || ns == d->S) &&
                  (count > 0.0 || ns == 1),
              "bn_fwd_apply: bad argument (count <= 0 reads the count row of reduced sums: ns must be 1)");
  VFD_REQUIRE(!running_mean == !running_var, "bn_fwd_apply: running mean / var must come together");
  VFD_REQUIRE(!d->nhwc || ns == 1, "bn_fwd_apply: channels-last takes reduced sums (vfd_bn_sum, ns = 1)");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_BN_FWD, s);
  if (d->nhwc) {
    unsigned char* mk = d->relu ? relu_mask : nullptr;
    if (d->dtype == 1)
      bn_apply_nhwc_k<__bf16><<<dim3(nh_apply_blocks(d), G), BN_THREADS, 0, s>>>(
          *d, (const __bf16*)x, (const __bf16*)residual, sums, count, gamma, beta, (__bf16*)y, mean, invstd,
          running_mean, running_var, num_batches_tracked, mk);
    else
      bn_apply_nhwc_k<float><<<dim3(nh_apply_blocks(d), G), BN_THREADS, 0, s>>>(
          *d, (const float*)x, (const float*)residual, sums, count, gamma, beta, (float*)y, mean, invstd, running_mean,
          running_var, num_batches_tracked, mk);
    return fail_launch("bn_fwd_apply");
  }
  if (d->dtype == 1)
    bn_apply_k<__bf16><<<dim3(d->S, d->C, G), BN_THREADS, 0, s>>>(*d, (const __bf16*)x, (const __bf16*)residual, sums, ns,
                                                               count, gamma, beta, (__bf16*)y, mean, invstd, running_mean,
                                                               running_var, num_batches_tracked,
                                                               d->relu ? relu_mask : nullptr);
  else
    bn_apply_k<float><<<dim3(d->S, d->C, G), BN_THREADS, 0, s>>>(*d, (const float*)x, (const float*)residual, sums, ns,
                                                              count, gamma, beta, (float*)y, mean, invstd, running_mean,
                                                              running_var, num_batches_tracked,
                                                              d->relu ? relu_mask : nullptr);
  return fail_launch("bn_fwd_apply");
}

int vfd_bn_bwd_stats(const vfd_bn_desc* d, const void* g, const void* y, const void* x, const float* mean,
                     double* partial, void* stream) {
  if (int e = bn_check(d, "bn_bwd_stats")) return e;
  const int G = d->groups > 1 ? d->groups : 1;
  VFD_REQUIRE(g && x && mean && partial && (y || !d->relu), "bn_bwd_stats: null argument");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_BN_BWD, s);
  if (d->nhwc) {
    if (d->dtype == 1)
      bn_bwd_stats_nhwc_k<__bf16><<<dim3(d->S, G), BN_THREADS, 0, s>>>(*d, (const __bf16*)g, (const __bf16*)y,
                                                              (const __bf16*)x, mean, partial);
    else
      bn_bwd_stats_nhwc_k<float><<<dim3(d->S, G), BN_THREADS, 0, s>>>(*d, (const float*)g, (const float*)y, (const float*)x,
                                                             mean, partial);
    return fail_launch("bn_bwd_stats");
  }
  if (d->dtype == 1)
    bn_bwd_stats_k<__bf16><<<dim3(d->S, d->C, G), BN_THREADS, 0, s>>>(*d, (const __bf16*)g, (const __bf16*)y,
                                                                   (const __bf16*)x, mean, partial);
  else
    bn_bwd_stats_k<float><<<dim3(d->S, d->C, G), BN_THREADS, 0, s>>>(*d, (const float*)g, (const float*)y,
                                                                  (const float*)x, mean, partial);
  return fail_launch("bn_bwd_stats");
}

int vfd_bn_bwd_apply(const vfd_bn_desc* d, const void* g, const void* y, const void* x, const double* sums,
                     int ns, double count, const float* gamma, const float* mean, const float* invstd, void* dx,
                     void* dresidual, float* dgamma, float* dbeta, void* stream) {
  if (int e = bn_check(d, "bn_bwd_apply")) return e;
  const int G = d->groups > 1 ? d->groups : 1;
  VFD_REQUIRE(g && x && sums && gamma && mean && invstd && (y || !d->relu) && (ns == 1 || ns == d->S) &&
                  (count > 0.0 || ns == 1),
              "bn_bwd_apply: bad argument (count <= 0 reads the count row of reduced sums: ns must be 1)");
  VFD_REQUIRE(!d->nhwc || ns == 1, "bn_bwd_apply: channels-last takes reduced sums (vfd_bn_sum, ns = 1)");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_BN_BWD, s);
  if (d->nhwc) {
    if (d->dtype == 1)
      bn_bwd_apply_nhwc_k<__bf16><<<dim3(nh_apply_blocks(d), G), BN_THREADS, 0, s>>>(
          *d, (const __bf16*)g, (const __bf16*)y, (const __bf16*)x, sums, count, gamma, mean, invstd, (__bf16*)dx,
          (__bf16*)dresidual, dgamma, dbeta);
    else
      bn_bwd_apply_nhwc_k<float><<<dim3(nh_apply_blocks(d), G), BN_THREADS, 0, s>>>(
          *d, (const float*)g, (const float*)y, (const float*)x, sums, count, gamma, mean, invstd, (float*)dx,
          (float*)dresidual, dgamma, dbeta);
    return fail_launch("bn_bwd_apply");
  }
  if (d->dtype == 1)
    bn_bwd_apply_k<__bf16><<<dim3(d->S, d->C, G), BN_THREADS, 0, s>>>(*d, (const __bf16*)g, (const __bf16*)y,
                                                                   (const __bf16*)x, sums, ns, count, gamma, mean, invstd,
                                                                   (__bf16*)dx, (__bf16*)dresidual, dgamma, dbeta);
  else
    bn_bwd_apply_k<float><<<dim3(d->S, d->C, G), BN_THREADS, 0, s>>>(*d, (const float*)g, (const float*)y,
                                                                  (const float*)x, sums, ns, count, gamma, mean, invstd,
                                                                  (float*)dx, (float*)dresidual, dgamma, dbeta);
  return fail_launch("bn_bwd_apply");
}

int vfd_bn1_fits(const vfd_bn_desc* d) {
  if (!d || d->N <= 0 || d->C <= 0 || d->HW <= 0 || (long long)d->N * d->HW > (long long)BN1_MAX) return 0;
  if (d->groups < 0 || d->groups > 64) return 0;
  // groups: the NCHW one-launch kernels loop over them; channels-last maps take the split path
  return d->nhwc ? 0 : 1;
}

int vfd_bn1_fwd(const vfd_bn_desc* d, const void* x, const void* residual, const float* gamma, const float* beta,
                void* y, float* mean, float* invstd, float* running_mean, float* running_var,
                long long* num_batches_tracked, unsigned char* relu_mask, void* stream) {
  VFD_REQUIRE(vfd_bn1_fits(d), "bn1_fwd: channel larger than %u elements", BN1_MAX);
  VFD_REQUIRE(x && gamma && beta && y && mean && invstd && !running_mean == !running_var, "bn1_fwd: bad argument");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_BN_FWD, s);
  if (d->dtype == 1)
    bn1_fwd_k<__bf16><<<d->C, BN1_THREADS, 0, s>>>(*d, (const __bf16*)x, (const __bf16*)residual, gamma, beta,
                                                   (__bf16*)y, mean, invstd, running_mean, running_var,
                                                   num_batches_tracked, d->relu ? relu_mask : nullptr);
  else
    bn1_fwd_k<float><<<d->C, BN1_THREADS, 0, s>>>(*d, (const float*)x, (const float*)residual, gamma, beta, (float*)y,
                                                  mean, invstd, running_mean, running_var, num_batches_tracked,
                                                  d->relu ? relu_mask : nullptr);
  return fail_launch("bn1_fwd");
}

int vfd_bn1_bwd(const vfd_bn_desc* d, const void* g, const void* y, const void* x, const float* gamma,
                const float* mean, const float* invstd, void* dx, void* dresidual, float* dgamma, float* dbeta,
                void* stream) {
  VFD_REQUIRE(vfd_bn1_fits(d), "bn1_bwd: channel larger than %u elements", BN1_MAX);
  VFD_REQUIRE(g && x && gamma && mean && invstd && (y || !d->relu), "bn1_bwd: bad argument");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_BN_BWD, s);
  if (d->dtype == 1)
    bn1_bwd_k<__bf16><<<d->C, BN1_THREADS, 0, s>>>(*d, (const __bf16*)g, (const __bf16*)y, (const __bf16*)x, gamma,
                                                   mean, invstd, (__bf16*)dx, (__bf16*)dresidual, dgamma, dbeta);
  else
    bn1_bwd_k<float><<<d->C, BN1_THREADS, 0, s>>>(*d, (const float*)g, (const float*)y, (const float*)x, gamma, mean,
                                                  invstd, (float*)dx, (float*)dresidual, dgamma, dbeta);
  return fail_launch("bn1_bwd");
}

}  // extern "C"
