// Reflect padding by one pixel (nn.Conv2d(padding_mode='reflect', padding=1): the decoders'
// 3x3 convs, network/blocks.py conv2d blocks) for NCHW fp32 or bf16 maps (config 3's autocast;
// arithmetic in fp32, one rounding per output), forward and backward, alone
// or fused with the ELU [+ nearest 2x upsample] in front of it (elu_up_pad_*: the plain pad is
// the <UP = 0, ACT = false> instance).  The backward is a gather: every input pixel sums its
// (up to four) padded copies in a fixed order, so it needs no atomics and is deterministic
// (ATen's reflection_pad2d backward scatters with atomics).
#include "vfd_common.h"

namespace vfd {

__device__ __forceinline__ int rp_src(int i, int n) {       // padded index -> source index
  return i == 0 ? 1 : (i == n + 1 ? n - 2 : i - 1);
}

// Backward of LeakyReLU(slope) followed by the one-pixel reflect pad, channels-last (the fused
// reduce_dim convs' outputs, projconv.hip / padconv.hip): gp[n][y][x][c] = (sum of the copies of
// g at pixel (y, x)) * (out[n][y+1][x+1][c] > 0 ? 1 : slope); float4 lanes over channels.
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void lrelu_pad_bwd_nhwc_k(const TI* __restrict__ g, const TI* __restrict__ out,
                                                            TO* __restrict__ gp, long long n_img, int h, int w,
                                                            int c4, float slope) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;       // (pixel, channel quad) of image blockIdx.y
  if (j >= h * w * c4) return;
  const long long n = blockIdx.y;
  const int pix = j / c4, q = j - pix * c4;
  const int yy = pix / w, x = pix - yy * w;
  const int wo = w + 2;
  const size_t i = (size_t)n * h * w * c4 + j;
  int rows[3], cols[3], nr, nc;
  pad_sets(yy, h, true, rows, &nr);
  pad_sets(x, w, true, cols, &nc);
  const TI* gb = g + ((size_t)n * (h + 2) * wo * c4 + q) * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int a = 0; a < nr; ++a)
    for (int b = 0; b < nc; ++b) {
      const float4 v = ld4(gb + ((size_t)rows[a] * wo + cols[b]) * c4 * 4);
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
  const float4 o = ld4(out + (((n * (h + 2) + yy + 1) * wo + x + 1) * c4 + q) * 4);
  s.x *= o.x > 0.f ? 1.f : slope;
  s.y *= o.y > 0.f ? 1.f : slope;
  s.z *= o.z > 0.f ? 1.f : slope;
  s.w *= o.w > 0.f ? 1.f : slope;
  st4(gp + i * 4, s);
}


// ELU(alpha 1) [+ nearest 2x upsample] + one-pixel reflect pad, NCHW: the decoders' chain
// conv -> ELU -> upsample -> (next conv's) reflect pad (fusion_depthnet.py:97-145 conv2d blocks,
// blocks.py upsample) in one pass from the conv's pre-activation y [planes, h, w] to the padded
// input of the next conv [planes, Hu + 2, Wu + 2] (Hu = 2h or h).  out = elu(y) = expm1(y) for
// y <= 0 (ATen's elu formula).  A thread writes EPT consecutive outputs of the flat padded plane
// (one 16-B store when the plane size allows) for PPT planes (grid.y = plane groups), so the
// index arithmetic is paid once per PPT * EPT outputs.
constexpr int EPT = 4, PPT = 4;
__device__ __forceinline__ float elu1(float v) { return v <= 0.f ? expm1f(v) : v; }

template <int UP, bool ACT, typename T>
__global__ __launch_bounds__(256) void elu_up_pad_fwd_k(const T* __restrict__ y, T* __restrict__ out,
                                                        long long planes, int h, int w) {
  const int Hu = h << UP, Wu = w << UP;
  const int ho = Hu + 2, wo = Wu + 2, hwo = ho * wo;
  const int j0 = (blockIdx.x * blockDim.x + threadIdx.x) * EPT;   // first flat output of the plane
  if (j0 >= hwo) return;
  int src[EPT];
  int Y = j0 / wo, X = j0 - Y * wo;
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    src[e] = (rp_src(Y, Hu) >> UP) * w + (rp_src(X, Wu) >> UP);
    if (++X == wo) { X = 0; ++Y; }
  }
  const bool vec = (hwo % EPT) == 0;                          // every thread's 4 outputs in one plane row-run
  const long long p0 = (long long)blockIdx.y * PPT;
#pragma unroll
  for (int q = 0; q < PPT; ++q) {
    const long long p = p0 + q;
    if (p >= planes) break;
    const T* yp = y + p * h * w;
    float v[EPT];
#pragma unroll
    for (int e = 0; e < EPT; ++e) v[e] = ACT ? elu1(ld1(yp + src[e])) : ld1(yp + src[e]);
    T* op = out + p * hwo + j0;
    if (vec) {
      st4(op, make_float4(v[0], v[1], v[2], v[3]));
    } else {
#pragma unroll
      for (int e = 0; e < EPT; ++e)
        if (j0 + e < hwo) st1(op + e, v[e]);
    }
  }
}

// Its backward: dy = elu'(y) * (sum over the up-block's pixels of their reflect copies in g).
// The padded rows covering the block {2sy, 2sy+1} are 2sy+1, 2sy+2 plus a mirror row when a
// block pixel sits at 1 or Hu-2 (the rows of pad_sets of each pixel; the sets are disjoint),
// likewise the columns: a fixed-order gather of <= 4 x 4 values, no atomics.  ELU' from the
// output as ATen's elu_backward (is_result): out <= 0 ? g * (out + 1) : g.  A thread owns EPT
// consecutive pixels of a row (16-B y / dy accesses when w % 4 == 0) for PPT planes.
struct EupIdx {
  int a, b, ma, mb;           // padded rows/cols: a, b (up only), mirrors of pixels 1 / n-2
  float fma, fmb;             // 1 when that mirror exists (absent ones alias `a` and weigh 0)
};
template <int UP>
__device__ __forceinline__ EupIdx eup_idx(int s, int n) {
  const int Nu = n << UP, lo = s << UP, hi = lo + UP;        // the block's pixels lo..hi
  EupIdx r;
  r.a = lo + 1;
  r.b = lo + 2;
  const bool m1 = lo <= 1 && hi >= 1, m2 = lo <= Nu - 2 && hi >= Nu - 2;
  r.fma = m1 ? 1.f : 0.f;
  r.ma = m1 ? 0 : r.a;
  r.fmb = m2 ? 1.f : 0.f;
  r.mb = m2 ? Nu + 1 : r.a;
  return r;
}

template <int UP, typename T>
__device__ __forceinline__ float eup_row(const T* __restrict__ gr, const EupIdx& C) {
  float t = ld1(gr + C.a);
  if (UP) t += ld1(gr + C.b);
  if (C.fma != 0.f || C.fmb != 0.f) t = (t + C.fma * ld1(gr + C.ma)) + C.fmb * ld1(gr + C.mb);
  return t;
}

// psum (optional): psum[p * gridDim.x + blockIdx.x] = the block's sum of dy over plane p (the
// conv bias gradient's partials, summed in a fixed order by the caller: no ATen reduction pass)
template <int UP, bool ACT, typename T>
__global__ __launch_bounds__(256) void elu_up_pad_bwd_k(const T* __restrict__ g, const T* __restrict__ y,
                                                        T* __restrict__ dy, long long planes, int h, int w,
                                                        float* __restrict__ psum) {
  __shared__ float red[256 / 64];
  const int Hu = h << UP, Wu = w << UP;
  const int wo = Wu + 2;
  const int wq = (w + EPT - 1) / EPT;                        // thread groups per row
  const int j0 = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = j0 < h * wq;                             // dead threads still join the block sums
  const int j = live ? j0 : 0;
  const int sy = j / wq, sx0 = (j - sy * wq) * EPT;
  const EupIdx R = eup_idx<UP>(sy, h);
  const bool rmir = R.fma != 0.f || R.fmb != 0.f;           // rare: border rows
  EupIdx C[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) C[e] = eup_idx<UP>(min(sx0 + e, w - 1), w);
  const bool vec = (w % EPT) == 0;
  const long long p0 = (long long)blockIdx.y * PPT;
#pragma unroll 1
  for (int q = 0; q < PPT; ++q) {
    const long long p = p0 + q;
    if (p >= planes) break;
    const T* gp = g + p * (Hu + 2) * wo;
    const T* ga = gp + (size_t)R.a * wo;
    const T* gb = gp + (size_t)R.b * wo;
    float s[EPT];
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      s[e] = eup_row<UP>(ga, C[e]);
      if (UP) s[e] += eup_row<UP>(gb, C[e]);
      if (rmir) {
        s[e] += R.fma * eup_row<UP>(gp + (size_t)R.ma * wo, C[e]);
        s[e] += R.fmb * eup_row<UP>(gp + (size_t)R.mb * wo, C[e]);
      }
    }
    const size_t o = p * h * w + (size_t)sy * w + sx0;
    float v[EPT] = {};
    if (!ACT) {
    } else if (vec) {
      const float4 t = ld4(y + o);
      v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else {
#pragma unroll
      for (int e = 0; e < EPT; ++e) v[e] = ld1(y + o + (sx0 + e < w ? e : 0));
    }
    float r[EPT];
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const float ov = elu1(v[e]);
      r[e] = !ACT ? s[e] : (ov <= 0.f ? s[e] * (ov + 1.f) : s[e]);
    }
    if (live) {
      if (vec) {
        st4(dy + o, make_float4(r[0], r[1], r[2], r[3]));
      } else {
#pragma unroll
        for (int e = 0; e < EPT; ++e)
          if (sx0 + e < w) st1(dy + o + e, r[e]);
      }
    }
    if (psum) {                                              // block-uniform branch
      float t = 0.f;
#pragma unroll
      for (int e = 0; e < EPT; ++e) t += (live && sx0 + e < w) ? r[e] : 0.f;
      t = wave_sum(t);
      __syncthreads();
      if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
      __syncthreads();
      if (threadIdx.x == 0) psum[p * gridDim.x + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
    }
  }
}

// ---- channels-last forms (config 3's bf16 decoders keep their maps NHWC, so MIOpen's convolutions
// run without their NCHW <-> NHWC transposes).  Same per-channel arithmetic as the NCHW kernels:
// thread = (padded output pixel | source pixel, channel quad), 8-B bf16 / 16-B fp32 accesses.
template <int UP, bool ACT, typename T>
__global__ __launch_bounds__(256) void elu_up_pad_fwd_nhwc_k(const T* __restrict__ y, T* __restrict__ out,
                                                             long long n_img, int h, int w, int Q) {
  const int Hu = h << UP, Wu = w << UP;
  const int ho = Hu + 2, wo = Wu + 2;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_img * ho * wo * Q) return;
  const int q = (int)(i % Q);
  const long long pix = i / Q;
  const int X = (int)(pix % wo);
  const long long r = pix / wo;
  const int Y = (int)(r % ho);
  const long long n = r / ho;
  const int sy = rp_src(Y, Hu) >> UP, sx = rp_src(X, Wu) >> UP;
  float4 v = ld4(y + ((n * h + sy) * w + sx) * (4LL * Q) + 4 * q);
  if (ACT) {
    v.x = elu1(v.x);
    v.y = elu1(v.y);
    v.z = elu1(v.z);
    v.w = elu1(v.w);
  }
  st4(out + pix * (4LL * Q) + 4 * q, v);
}

template <int UP, typename T>
__device__ __forceinline__ float4 eup_row_nhwc(const T* __restrict__ gr, const EupIdx& C, int ld) {
  // eup_row's order per channel: a (+ b) then (+ fma * ma) + fmb * mb
  float4 t = ld4(gr + (size_t)C.a * ld);
  if (UP) {
    const float4 b = ld4(gr + (size_t)C.b * ld);
    t.x += b.x; t.y += b.y; t.z += b.z; t.w += b.w;
  }
  if (C.fma != 0.f || C.fmb != 0.f) {
    const float4 ma = ld4(gr + (size_t)C.ma * ld), mb = ld4(gr + (size_t)C.mb * ld);
    t.x = (t.x + C.fma * ma.x) + C.fmb * mb.x;
    t.y = (t.y + C.fma * ma.y) + C.fmb * mb.y;
    t.z = (t.z + C.fma * ma.z) + C.fmb * mb.z;
    t.w = (t.w + C.fma * ma.w) + C.fmb * mb.w;
  }
  return t;
}

// part (optional, [gridDim.x][4 Q]): the block's per-channel sums of dy (conv bias partials; a block
// covers whole pixels: 256 / Q of them), summed over blocks by the caller
template <int UP, bool ACT, typename T>
__global__ __launch_bounds__(256) void elu_up_pad_bwd_nhwc_k(const T* __restrict__ g, const T* __restrict__ y,
                                                             T* __restrict__ dy, long long n_img, int h, int w, int Q,
                                                             float* __restrict__ part) {
  __shared__ float4 red[256];
  const int Hu = h << UP, Wu = w << UP;
  const int wo = Wu + 2, ld = 4 * Q;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = i < n_img * h * w * Q;
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (live) {
    const int q = (int)(i % Q);
    const long long pix = i / Q;
    const int sx = (int)(pix % w);
    const long long rr = pix / w;
    const int sy = (int)(rr % h);
    const long long n = rr / h;
    const EupIdx R = eup_idx<UP>(sy, h), C = eup_idx<UP>(sx, w);
    const T* gp = g + (size_t)n * (Hu + 2) * wo * ld + 4 * q;
    // per row: eup_row over the columns; rows a (+ b) then the mirrors, as elu_up_pad_bwd_k
    float4 s = eup_row_nhwc<UP>(gp + (size_t)R.a * wo * ld, C, ld);
    if (UP) {
      const float4 t = eup_row_nhwc<UP>(gp + (size_t)R.b * wo * ld, C, ld);
      s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    }
    if (R.fma != 0.f || R.fmb != 0.f) {
      const float4 ta = eup_row_nhwc<UP>(gp + (size_t)R.ma * wo * ld, C, ld);
      s.x += R.fma * ta.x; s.y += R.fma * ta.y; s.z += R.fma * ta.z; s.w += R.fma * ta.w;
      const float4 tb = eup_row_nhwc<UP>(gp + (size_t)R.mb * wo * ld, C, ld);
      s.x += R.fmb * tb.x; s.y += R.fmb * tb.y; s.z += R.fmb * tb.z; s.w += R.fmb * tb.w;
    }
    r = s;
    const size_t o = (size_t)pix * ld + 4 * q;
    if (ACT) {
      const float4 v = ld4(y + o);
      float ov;
      ov = elu1(v.x); r.x = ov <= 0.f ? s.x * (ov + 1.f) : s.x;
      ov = elu1(v.y); r.y = ov <= 0.f ? s.y * (ov + 1.f) : s.y;
      ov = elu1(v.z); r.z = ov <= 0.f ? s.z * (ov + 1.f) : s.z;
      ov = elu1(v.w); r.w = ov <= 0.f ? s.w * (ov + 1.f) : s.w;
    }
    st4(dy + o, r);
  }
  if (part) {                                  // block-uniform: fixed-order sums over the block's pixels
    red[threadIdx.x] = r;
    __syncthreads();
    if (threadIdx.x < Q) {
      float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int k = threadIdx.x; k < 256; k += Q) {
        t.x += red[k].x; t.y += red[k].y; t.z += red[k].z; t.w += red[k].w;
      }
      *reinterpret_cast<float4*>(part + (size_t)blockIdx.x * ld + 4 * threadIdx.x) = t;
    }
  }
}

}  // namespace vfd

using namespace vfd;

extern "C" {

int vfd_reflect_pad1_fwd(const void* x, void* y, long long planes, int h, int w, int dtype, void* stream) {
  VFD_REQUIRE(x && y && planes > 0 && h >= 2 && w >= 2 && (long long)(h + 2) * (w + 2) < (1LL << 31) &&
                  (dtype == 0 || dtype == 1),
              "reflect_pad1: bad arguments (h, w >= 2)");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_REFLECT_PAD, s);
  VFD_REQUIRE(planes / PPT < 65535, "reflect_pad1: too many planes");
  const dim3 grid((unsigned)(((h + 2) * (w + 2) + 256 * EPT - 1) / (256 * EPT)), (unsigned)((planes + PPT - 1) / PPT));
  if (dtype == 1) elu_up_pad_fwd_k<0, false><<<grid, 256, 0, s>>>((const __bf16*)x, (__bf16*)y, planes, h, w);
  else elu_up_pad_fwd_k<0, false><<<grid, 256, 0, s>>>((const float*)x, (float*)y, planes, h, w);
  return fail_launch("reflect_pad1_fwd");
}

int vfd_reflect_pad1_bwd(const void* g, void* dx, long long planes, int h, int w, int dtype, void* stream) {
  VFD_REQUIRE(g && dx && planes > 0 && h >= 2 && w >= 2 && (long long)(h + 2) * (w + 2) < (1LL << 31) &&
                  (dtype == 0 || dtype == 1),
              "reflect_pad1: bad arguments (h, w >= 2)");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_REFLECT_PAD, s);
  VFD_REQUIRE(planes / PPT < 65535, "reflect_pad1: too many planes");
  const dim3 grid((unsigned)((h * ((w + EPT - 1) / EPT) + 255) / 256), (unsigned)((planes + PPT - 1) / PPT));
  if (dtype == 1)
    elu_up_pad_bwd_k<0, false><<<grid, 256, 0, s>>>((const __bf16*)g, (const __bf16*)nullptr, (__bf16*)dx, planes, h,
                                                    w, nullptr);
  else
    elu_up_pad_bwd_k<0, false><<<grid, 256, 0, s>>>((const float*)g, (const float*)nullptr, (float*)dx, planes, h, w,
                                                    nullptr);
  return fail_launch("reflect_pad1_bwd");
}

int vfd_lrelu_pad1_bwd_nhwc(const float* g, const float* out, float* gp, long long n_img, int h, int w, int C,
                            float slope, void* stream) {
  VFD_REQUIRE(g && out && gp && n_img > 0 && h >= 2 && w >= 2 && C > 0 && C % 4 == 0,
              "lrelu_pad1_bwd_nhwc: bad arguments (h, w >= 2, C %% 4 == 0)");
  VFD_REQUIRE((((uintptr_t)g | (uintptr_t)out | (uintptr_t)gp) & 15) == 0, "lrelu_pad1_bwd_nhwc: 16-B alignment");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_REFLECT_PAD, s);
  VFD_REQUIRE(n_img < 65536 && (long long)h * w * C < (1LL << 31), "lrelu_pad1_bwd_nhwc: too large");
  const dim3 grid((unsigned)(((long long)h * w * (C / 4) + 255) / 256), (unsigned)n_img);
  lrelu_pad_bwd_nhwc_k<float, float><<<grid, 256, 0, s>>>(g, out, gp, n_img, h, w, C / 4, slope);
  return fail_launch("lrelu_pad1_bwd_nhwc");
}

int vfd_lrelu_pad1_bwd_nhwc_t(const void* g, const void* out, void* gp, long long n_img, int h, int w, int C,
                              float slope, int dtype_in, int dtype_out, void* stream) {
  VFD_REQUIRE(g && out && gp && n_img > 0 && h >= 2 && w >= 2 && C > 0 && C % 4 == 0 && (dtype_in == 0 || dtype_in == 1) &&
                  (dtype_out == 0 || dtype_out == 1),
              "lrelu_pad1_bwd_nhwc_t: bad arguments (h, w >= 2, C %% 4 == 0, dtypes 0 fp32 / 1 bf16)");
  VFD_REQUIRE((((uintptr_t)g | (uintptr_t)out | (uintptr_t)gp) & 7) == 0, "lrelu_pad1_bwd_nhwc_t: 8-B alignment");
  VFD_REQUIRE(n_img < 65536 && (long long)h * w * C < (1LL << 31), "lrelu_pad1_bwd_nhwc_t: too large");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_REFLECT_PAD, s);
  const dim3 grid((unsigned)(((long long)h * w * (C / 4) + 255) / 256), (unsigned)n_img);
  if (dtype_in == 0 && dtype_out == 0)
    lrelu_pad_bwd_nhwc_k<float, float><<<grid, 256, 0, s>>>((const float*)g, (const float*)out, (float*)gp, n_img, h, w, C / 4, slope);
  else if (dtype_in == 0)
    lrelu_pad_bwd_nhwc_k<float, __bf16><<<grid, 256, 0, s>>>((const float*)g, (const float*)out, (__bf16*)gp, n_img, h, w, C / 4, slope);
  else if (dtype_out == 0)
    lrelu_pad_bwd_nhwc_k<__bf16, float><<<grid, 256, 0, s>>>((const __bf16*)g, (const __bf16*)out, (float*)gp, n_img, h, w, C / 4, slope);
  else
    lrelu_pad_bwd_nhwc_k<__bf16, __bf16><<<grid, 256, 0, s>>>((const __bf16*)g, (const __bf16*)out, (__bf16*)gp, n_img, h, w, C / 4, slope);
  return fail_launch("lrelu_pad1_bwd_nhwc_t");
}

int vfd_elu_up_pad1_fwd(const void* y, void* out, long long planes, int h, int w, int up, int dtype, void* stream) {
  VFD_REQUIRE(y && out && planes > 0 && planes / PPT < 65535 && h >= 1 && w >= 1 && (up == 0 || up == 1) && (h << up) >= 2 &&
                  (dtype == 0 || dtype == 1) &&
                  (w << up) >= 2 && (long long)((h << up) + 2) * ((w << up) + 2) < (1LL << 31),
              "elu_up_pad1: bad arguments (up in {0, 1}, padded side >= 2)");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_ELU_PAD, s);
  const unsigned gx = (unsigned)((((h << up) + 2) * ((w << up) + 2) + 256 * EPT - 1) / (256 * EPT));
  const dim3 grid(gx, (unsigned)((planes + PPT - 1) / PPT));
  if (dtype == 1) {
    if (up) elu_up_pad_fwd_k<1, true><<<grid, 256, 0, s>>>((const __bf16*)y, (__bf16*)out, planes, h, w);
    else elu_up_pad_fwd_k<0, true><<<grid, 256, 0, s>>>((const __bf16*)y, (__bf16*)out, planes, h, w);
  } else {
    if (up) elu_up_pad_fwd_k<1, true><<<grid, 256, 0, s>>>((const float*)y, (float*)out, planes, h, w);
    else elu_up_pad_fwd_k<0, true><<<grid, 256, 0, s>>>((const float*)y, (float*)out, planes, h, w);
  }
  return fail_launch("elu_up_pad1_fwd");
}

int vfd_elu_up_pad1_bwd_blocks(int h, int w) { return (h * ((w + EPT - 1) / EPT) + 255) / 256; }

int vfd_elu_up_pad1_bwd(const void* g, const void* y, void* dy, long long planes, int h, int w, int up,
                        float* psum, int dtype, void* stream) {
  VFD_REQUIRE(g && y && dy && planes > 0 && planes / PPT < 65535 && h >= 1 && w >= 1 && (up == 0 || up == 1) && (h << up) >= 2 &&
                  (dtype == 0 || dtype == 1) &&
                  (w << up) >= 2 && (long long)((h << up) + 2) * ((w << up) + 2) < (1LL << 31),
              "elu_up_pad1: bad arguments (up in {0, 1}, padded side >= 2)");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_ELU_PAD, s);
  const dim3 grid((unsigned)((h * ((w + EPT - 1) / EPT) + 255) / 256), (unsigned)((planes + PPT - 1) / PPT));
  if (dtype == 1) {
    const __bf16 *gb = (const __bf16*)g, *yb = (const __bf16*)y;
    if (up) elu_up_pad_bwd_k<1, true><<<grid, 256, 0, s>>>(gb, yb, (__bf16*)dy, planes, h, w, psum);
    else elu_up_pad_bwd_k<0, true><<<grid, 256, 0, s>>>(gb, yb, (__bf16*)dy, planes, h, w, psum);
  } else {
    const float *gf = (const float*)g, *yf = (const float*)y;
    if (up) elu_up_pad_bwd_k<1, true><<<grid, 256, 0, s>>>(gf, yf, (float*)dy, planes, h, w, psum);
    else elu_up_pad_bwd_k<0, true><<<grid, 256, 0, s>>>(gf, yf, (float*)dy, planes, h, w, psum);
  }
  return fail_launch("elu_up_pad1_bwd");
}

// channels-last [n_img, h, w, C] -> [n_img, Hu + 2, Wu + 2, C], C % 4 == 0 (act 0: the plain pad)
int vfd_elu_up_pad1_nhwc_fwd(const void* y, void* out, long long n_img, int h, int w, int C, int up, int act,
                             int dtype, void* stream) {
  VFD_REQUIRE(y && out && n_img > 0 && h >= 1 && w >= 1 && C > 0 && C % 4 == 0 && (up == 0 || up == 1) &&
                  (act == 0 || act == 1) && (dtype == 0 || dtype == 1) && (h << up) >= 2 && (w << up) >= 2 &&
                  (((uintptr_t)y | (uintptr_t)out) & (dtype ? 7 : 15)) == 0,
              "elu_up_pad1_nhwc: bad arguments (C %% 4 == 0, up in {0, 1}, padded side >= 2, aligned maps)");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(act ? K_ELU_PAD : K_REFLECT_PAD, s);
  const long long total = n_img * (long long)((h << up) + 2) * ((w << up) + 2) * (C / 4);
  const unsigned grid = (unsigned)((total + 255) / 256);
#define VFD_EUP_N(U, A, T) elu_up_pad_fwd_nhwc_k<U, A, T><<<grid, 256, 0, s>>>((const T*)y, (T*)out, n_img, h, w, C / 4)
  if (dtype == 1) {
    if (up) { if (act) VFD_EUP_N(1, true, __bf16); else VFD_EUP_N(1, false, __bf16); }
    else { if (act) VFD_EUP_N(0, true, __bf16); else VFD_EUP_N(0, false, __bf16); }
  } else {
    if (up) { if (act) VFD_EUP_N(1, true, float); else VFD_EUP_N(1, false, float); }
    else { if (act) VFD_EUP_N(0, true, float); else VFD_EUP_N(0, false, float); }
  }
#undef VFD_EUP_N
  return fail_launch("elu_up_pad1_nhwc_fwd");
}

int vfd_elu_up_pad1_nhwc_bwd_blocks(long long n_img, int h, int w, int C) {
  return (int)((n_img * h * w * (C / 4) + 255) / 256);
}

// y (act 1: the conv's pre-activation, channels-last [n_img, h, w, C]) may be NULL for act 0
int vfd_elu_up_pad1_nhwc_bwd(const void* g, const void* y, void* dy, long long n_img, int h, int w, int C, int up,
                             int act, float* part, int dtype, void* stream) {
  VFD_REQUIRE(g && dy && (y || !act) && n_img > 0 && h >= 1 && w >= 1 && C > 0 && C % 4 == 0 && 256 % (C / 4) == 0 &&
                  (up == 0 || up == 1) && (act == 0 || act == 1) && (dtype == 0 || dtype == 1) &&
                  (h << up) >= 2 && (w << up) >= 2 &&
                  (((uintptr_t)g | (uintptr_t)y | (uintptr_t)dy | (uintptr_t)part) & (dtype ? 7 : 15)) == 0,
              "elu_up_pad1_nhwc_bwd: bad arguments (C %% 4 == 0, C / 4 divides 256, up in {0, 1}, padded side >= 2, "
              "aligned maps)");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(act ? K_ELU_PAD : K_REFLECT_PAD, s);
  const unsigned grid = (unsigned)vfd_elu_up_pad1_nhwc_bwd_blocks(n_img, h, w, C);
#define VFD_EUPB_N(U, A, T) \
  elu_up_pad_bwd_nhwc_k<U, A, T><<<grid, 256, 0, s>>>((const T*)g, (const T*)y, (T*)dy, n_img, h, w, C / 4, part)
  if (dtype == 1) {
    if (up) { if (act) VFD_EUPB_N(1, true, __bf16); else VFD_EUPB_N(1, false, __bf16); }
    else { if (act) VFD_EUPB_N(0, true, __bf16); else VFD_EUPB_N(0, false, __bf16); }
  } else {
    if (up) { if (act) VFD_EUPB_N(1, true, float); else VFD_EUPB_N(1, false, float); }
    else { if (act) VFD_EUPB_N(0, true, float); else VFD_EUPB_N(0, false, float); }
  }
#undef VFD_EUPB_N
  return fail_launch("elu_up_pad1_nhwc_bwd");
}

}  // extern "C"
