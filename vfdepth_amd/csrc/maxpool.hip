// MaxPool2d(3, stride 2, padding 1) of the ResNet stem (torchvision / packnet ResnetEncoder,
// fusion_depthnet.py:24-36, fusion_posenet.py:22-35), NCHW fp32 or bf16 (config 3's autocast;
// compared and summed in fp32), forward and backward.
// The forward keeps the winning window position as one byte (ATen stores an int64 index: 8x the
// bytes); ties go to the first maximum in window scan order and NaN wins, as ATen's `val > max ||
// isnan(val)` does.  The backward is a gather: every input pixel sums the gradients of the (<= 4)
// output windows whose winner it is, in a fixed order (deterministic, no atomics).
#include "vfd_common.h"

namespace vfd {

template <typename T>
__global__ __launch_bounds__(256) void maxpool_fwd_k(const T* __restrict__ x, T* __restrict__ y,
                                                     uint8_t* __restrict__ arg, long long planes, int h, int w,
                                                     int ho, int wo) {
  // grid (cdiv(ho*wo, 256), planes): 32-bit index math inside a plane (64-bit division is a
  // long software sequence on CDNA and made this kernel ALU-bound)
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ho * wo) return;
  const int oy = j / wo, ox = j - oy * wo;
  for (long long p = blockIdx.y; p < planes; p += gridDim.y) {
    const size_t i = (size_t)p * ho * wo + j;
    const T* xp = x + (size_t)p * h * w;
    float v[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {                    // unconditional loads at clamped taps
      const int yy = min(max(2 * oy - 1 + k / 3, 0), h - 1), xx = min(max(2 * ox - 1 + k % 3, 0), w - 1);
      v[k] = ld1(xp + yy * w + xx);
    }
    float best = -INFINITY;
    int bi = 4;                                      // centre (always inside the image)
    bool first = true;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int yy = 2 * oy - 1 + k / 3, xx = 2 * ox - 1 + k % 3;
      const bool ok = yy >= 0 && yy < h && xx >= 0 && xx < w;
      if (ok && (first || v[k] > best || isnan(v[k]))) {
        best = v[k];
        bi = k;
        first = false;
      }
    }
    st1(y + i, best);
    arg[i] = (uint8_t)bi;
  }
}

// Four consecutive outputs per thread (wo % 4 == 0, w == 2 wo): each of the 3 window rows is one
// scalar (column 2 ox0 - 1) and two 16-B loads (columns 2 ox0 .. 2 ox0 + 7), 9 load instructions
// for 4 outputs instead of 36; the taps, their order and the selection are maxpool_fwd_k's.
template <typename T>
__global__ __launch_bounds__(256) void maxpool_fwd4_k(const T* __restrict__ x, T* __restrict__ y,
                                                      uint8_t* __restrict__ arg, long long planes, int h, int w,
                                                      int ho, int wo) {
  const int wq = wo / 4;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ho * wq) return;
  const int oy = j / wq, ox0 = (j - oy * wq) * 4;
  for (long long p = blockIdx.y; p < planes; p += gridDim.y) {
    const T* xp = x + (size_t)p * h * w;
    float r[3][9];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const T* row = xp + min(max(2 * oy - 1 + ky, 0), h - 1) * w;
      const float4 a = ld4(row + 2 * ox0);
      const float4 b = ld4(row + 2 * ox0 + 4);
      r[ky][0] = ld1(row + max(2 * ox0 - 1, 0));
      r[ky][1] = a.x; r[ky][2] = a.y; r[ky][3] = a.z; r[ky][4] = a.w;
      r[ky][5] = b.x; r[ky][6] = b.y; r[ky][7] = b.z; r[ky][8] = b.w;
    }
    float best4[4];
    unsigned code = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ox = ox0 + e;
      float best = -INFINITY;
      int bi = 4;
      bool first = true;
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int ky = k / 3, kx = k % 3;
        const int yy = 2 * oy - 1 + ky, xx = 2 * ox - 1 + kx;
        const bool ok = yy >= 0 && yy < h && xx >= 0 && xx < w;
        const float v = r[ky][2 * e + kx];
        if (ok && (first || v > best || isnan(v))) {
          best = v;
          bi = k;
          first = false;
        }
      }
      best4[e] = best;
      code |= (unsigned)bi << (8 * e);
    }
    const size_t i = (size_t)p * ho * wo + (size_t)oy * wo + ox0;
    st4(y + i, make_float4(best4[0], best4[1], best4[2], best4[3]));
    *reinterpret_cast<unsigned*>(arg + i) = code;
  }
}

// One thread per 2x2 input block (rows 2i, 2i+1; columns 2j, 2j+1): the block's pixels are covered
// by the output windows (i, j), (i, j+1), (i+1, j), (i+1, j+1) only (pixel 2i sits in window i's
// centre row, pixel 2i+1 in window i's last row and window i+1's first), so 4 gradient and 4 index
// loads serve 4 pixels; each pixel sums its winning windows in ATen's (row, column) order.
template <typename T>
__global__ __launch_bounds__(256) void maxpool_bwd_k(const T* __restrict__ g, const uint8_t* __restrict__ arg,
                                                     T* __restrict__ dx, long long planes, int h, int w, int ho,
                                                     int wo) {
  const int hb = (h + 1) / 2, wb = (w + 1) / 2;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= hb * wb) return;
  const int bi = j / wb, bj = j - bi * wb;               // == output row / column of window (i, j)
  const bool r1 = bi + 1 < ho, c1 = bj + 1 < wo;          // neighbouring windows exist
  const int o = bi * wo + bj;
  const int y0 = 2 * bi, x0 = 2 * bj;
  const bool y1in = y0 + 1 < h, x1in = x0 + 1 < w;
  for (long long p = blockIdx.y; p < planes; p += gridDim.y) {
    const T* gp = g + (size_t)p * ho * wo;
    const uint8_t* ap = arg + (size_t)p * ho * wo;
    // unconditional loads at clamped offsets; windows past the edge get index 255 (never wins)
    const int o01 = c1 ? o + 1 : o, o10 = r1 ? o + wo : o, o11 = (r1 && c1) ? o + wo + 1 : o;
    const int l00 = ap[o], l01 = ap[o01], l10 = ap[o10], l11 = ap[o11];
    const float g00 = ld1(gp + o), g01 = ld1(gp + o01), g10 = ld1(gp + o10), g11 = ld1(gp + o11);
    const int a00 = l00, a01 = c1 ? l01 : 255, a10 = r1 ? l10 : 255, a11 = (r1 && c1) ? l11 : 255;
    // window positions (ky * 3 + kx): pixel (2i, 2j) is (1,1) of (i,j); (2i, 2j+1) is (1,2) of
    // (i,j) and (1,0) of (i,j+1); (2i+1, 2j) is (2,1) of (i,j) and (0,1) of (i+1,j); (2i+1, 2j+1)
    // is (2,2) of (i,j), (2,0) of (i,j+1), (0,2) of (i+1,j) and (0,0) of (i+1,j+1)
    float d00 = 0.f, d01 = 0.f, d10 = 0.f, d11 = 0.f;
    if (a00 == 4) d00 += g00;
    if (a00 == 5) d01 += g00;
    if (a01 == 3) d01 += g01;
    if (a00 == 7) d10 += g00;
    if (a10 == 1) d10 += g10;
    if (a00 == 8) d11 += g00;
    if (a01 == 6) d11 += g01;
    if (a10 == 2) d11 += g10;
    if (a11 == 0) d11 += g11;
    T* dp = dx + (size_t)p * h * w + (size_t)y0 * w + x0;
    st1(dp, d00);
    if (x1in) st1(dp + 1, d01);
    if (y1in) {
      st1(dp + w, d10);
      if (x1in) st1(dp + w + 1, d11);
    }
  }
}

// ---- channels-last (config 3's bf16 encoders, layers.ResnetEncoder.use_channels_last): x [n][h][w][C],
// y / arg [n][ho][wo][C].  One thread per (output pixel, channel quad): every tap is one 4-channel
// load contiguous across the wave; the taps, their order and the selection are maxpool_fwd_k's,
// per channel.
template <typename T>
__global__ __launch_bounds__(256) void maxpool_nhwc_fwd_k(const T* __restrict__ x, T* __restrict__ y,
                                                          uint8_t* __restrict__ arg, int n, int C, int h, int w,
                                                          int ho, int wo) {
  // 32-bit index math (host-checked < 2^31 work items): 64-bit division is a long software sequence
  const unsigned Q = (unsigned)C >> 2;
  const unsigned total = (unsigned)n * ho * wo * Q;
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const unsigned q = t % Q;
    const unsigned pix = t / Q;                        // (img, oy, ox)
    const int ox = (int)(pix % (unsigned)wo);
    const unsigned r = pix / (unsigned)wo;
    const int oy = (int)(r % (unsigned)ho);
    const unsigned img = r / (unsigned)ho;
    const T* xp = x + (size_t)img * h * w * C + 4 * q;
    float best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int bi[4] = {4, 4, 4, 4};
    bool first[4] = {true, true, true, true};
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int yy = 2 * oy - 1 + k / 3, xx = 2 * ox - 1 + k % 3;
      if (yy < 0 || yy >= h || xx < 0 || xx >= w) continue;
      const float4 v4 = ld4(xp + ((size_t)yy * w + xx) * C);
      const float v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (first[e] || v[e] > best[e] || isnan(v[e])) {
          best[e] = v[e];
          bi[e] = k;
          first[e] = false;
        }
    }
    const size_t o = (size_t)pix * C + 4 * q;
    st4(y + o, make_float4(best[0], best[1], best[2], best[3]));
    *reinterpret_cast<uchar4*>(arg + o) = make_uchar4(bi[0], bi[1], bi[2], bi[3]);
  }
}

// channels-last backward: one thread per (2x2 input block, channel quad), maxpool_bwd_k's gather
template <typename T>
__global__ __launch_bounds__(256) void maxpool_nhwc_bwd_k(const T* __restrict__ g, const uint8_t* __restrict__ arg,
                                                          T* __restrict__ dx, int n, int C, int h, int w, int ho,
                                                          int wo) {
  const unsigned Q = (unsigned)C >> 2, hb = (h + 1) / 2, wb = (w + 1) / 2;
  const unsigned total = (unsigned)n * hb * wb * Q;
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const unsigned q = t % Q;
    const unsigned blk = t / Q;
    const int bj = (int)(blk % wb);
    const unsigned r = blk / wb;
    const int bi = (int)(r % hb);
    const unsigned img = r / hb;
    const bool r1 = bi + 1 < ho, c1 = bj + 1 < wo;
    const size_t base = (size_t)img * ho * wo;
    const size_t o00 = base + (size_t)bi * wo + bj;
    const size_t o01 = c1 ? o00 + 1 : o00, o10 = r1 ? o00 + wo : o00, o11 = (r1 && c1) ? o00 + wo + 1 : o00;
    const size_t cq = 4 * (size_t)q;
    const uchar4 l00 = *reinterpret_cast<const uchar4*>(arg + o00 * C + cq);
    const uchar4 l01 = *reinterpret_cast<const uchar4*>(arg + o01 * C + cq);
    const uchar4 l10 = *reinterpret_cast<const uchar4*>(arg + o10 * C + cq);
    const uchar4 l11 = *reinterpret_cast<const uchar4*>(arg + o11 * C + cq);
    const float4 g00 = ld4(g + o00 * C + cq), g01 = ld4(g + o01 * C + cq);
    const float4 g10 = ld4(g + o10 * C + cq), g11 = ld4(g + o11 * C + cq);
    const unsigned char A00[4] = {l00.x, l00.y, l00.z, l00.w}, A01[4] = {l01.x, l01.y, l01.z, l01.w};
    const unsigned char A10[4] = {l10.x, l10.y, l10.z, l10.w}, A11[4] = {l11.x, l11.y, l11.z, l11.w};
    const float G00[4] = {g00.x, g00.y, g00.z, g00.w}, G01[4] = {g01.x, g01.y, g01.z, g01.w};
    const float G10[4] = {g10.x, g10.y, g10.z, g10.w}, G11[4] = {g11.x, g11.y, g11.z, g11.w};
    float d00[4], d01[4], d10[4], d11[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int a00 = A00[e], a01 = c1 ? A01[e] : 255, a10 = r1 ? A10[e] : 255, a11 = (r1 && c1) ? A11[e] : 255;
      d00[e] = 0.f; d01[e] = 0.f; d10[e] = 0.f; d11[e] = 0.f;
      if (a00 == 4) d00[e] += G00[e];
      if (a00 == 5) d01[e] += G00[e];
      if (a01 == 3) d01[e] += G01[e];
      if (a00 == 7) d10[e] += G00[e];
      if (a10 == 1) d10[e] += G10[e];
      if (a00 == 8) d11[e] += G00[e];
      if (a01 == 6) d11[e] += G01[e];
      if (a10 == 2) d11[e] += G10[e];
      if (a11 == 0) d11[e] += G11[e];
    }
    const int y0 = 2 * bi, x0 = 2 * bj;
    T* dp = dx + (((size_t)img * h + y0) * w + x0) * C + cq;
    st4(dp, make_float4(d00[0], d00[1], d00[2], d00[3]));
    if (x0 + 1 < w) st4(dp + C, make_float4(d01[0], d01[1], d01[2], d01[3]));
    if (y0 + 1 < h) {
      st4(dp + (size_t)w * C, make_float4(d10[0], d10[1], d10[2], d10[3]));
      if (x0 + 1 < w) st4(dp + (size_t)w * C + C, make_float4(d11[0], d11[1], d11[2], d11[3]));
    }
  }
}

// The encoders' input normalisation (image - 0.45) / 0.225 (packnet ResnetEncoder), fused with the
// pose net's frame concatenation torch.cat([frame_a, frame_b], dim=channels) (fusion_posenet.py:
// 45-48): dst [n][c] = normalised (c < ca ? a[n][c] : b[n][c - ca]); one pass with 16-B accesses
// instead of cat + sub + div.  The same fp32 operations as ATen's GPU kernels (a tensor / CPU scalar
// division runs as a multiply by the fp32 reciprocal): bit-identical.
__global__ __launch_bounds__(256) void norm_cat_k(const float4* __restrict__ a, const float4* __restrict__ b,
                                                  float4* __restrict__ dst, long long n_img, int ca, int cb, int hw4) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int ct = ca + cb;
  if (i >= n_img * ct * hw4) return;
  const int p = (int)(i % hw4);
  const long long r = i / hw4;
  const int c = (int)(r % ct);
  const long long n = r / ct;
  const float4 v = c < ca ? a[(n * ca + c) * hw4 + p] : b[(n * cb + c - ca) * hw4 + p];
  const float rs = 1.0f / 0.225f;
  dst[i] = make_float4((v.x - 0.45f) * rs, (v.y - 0.45f) * rs, (v.z - 0.45f) * rs, (v.w - 0.45f) * rs);
}

}  // namespace vfd

template <typename T>
static int maxpool_fwd_launch(const T* x, T* y, uint8_t* arg, long long planes, int h, int w, hipStream_t s) {
  const int ho = (h - 1) / 2 + 1, wo = (w - 1) / 2 + 1;
  const unsigned gy = (unsigned)(planes < 65535 ? planes : 65535);
  const uintptr_t al = 4 * sizeof(T) - 1;
  if (wo % 4 == 0 && w == 2 * wo && (((uintptr_t)x | (uintptr_t)y) & al) == 0 && ((uintptr_t)arg & 3) == 0) {
    vfd::maxpool_fwd4_k<T><<<dim3((unsigned)((ho * (wo / 4) + 255) / 256), gy), 256, 0, s>>>(x, y, arg, planes, h, w, ho, wo);
  } else {
    vfd::maxpool_fwd_k<T><<<dim3((unsigned)((ho * wo + 255) / 256), gy), 256, 0, s>>>(x, y, arg, planes, h, w, ho, wo);
  }
  return vfd::fail_launch("maxpool3s2_fwd");
}

extern "C" {

int vfd_maxpool3s2_fwd(const void* x, void* y, uint8_t* arg, long long planes, int h, int w, int dtype, void* stream) {
  VFD_REQUIRE(x && y && arg && planes > 0 && h > 0 && w > 0 && (long long)h * w < (1LL << 31) && (dtype == 0 || dtype == 1),
              "maxpool3s2: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  vfd::ProfScope ps(vfd::K_MAXPOOL, s);
  if (dtype == 1) return maxpool_fwd_launch((const __bf16*)x, (__bf16*)y, arg, planes, h, w, s);
  return maxpool_fwd_launch((const float*)x, (float*)y, arg, planes, h, w, s);
}

int vfd_maxpool3s2_bwd(const void* g, const uint8_t* arg, void* dx, long long planes, int h, int w, int dtype,
                       void* stream) {
  VFD_REQUIRE(g && arg && dx && planes > 0 && h > 0 && w > 0 && (long long)h * w < (1LL << 31) && (dtype == 0 || dtype == 1),
              "maxpool3s2: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  vfd::ProfScope ps(vfd::K_MAXPOOL, s);
  const int ho = (h - 1) / 2 + 1, wo = (w - 1) / 2 + 1;
  const unsigned gy = (unsigned)(planes < 65535 ? planes : 65535);
  const int nblk2 = ((h + 1) / 2) * ((w + 1) / 2);
  const dim3 grid((unsigned)((nblk2 + 255) / 256), gy);
  if (dtype == 1)
    vfd::maxpool_bwd_k<__bf16><<<grid, 256, 0, s>>>((const __bf16*)g, arg, (__bf16*)dx, planes, h, w, ho, wo);
  else
    vfd::maxpool_bwd_k<float><<<grid, 256, 0, s>>>((const float*)g, arg, (float*)dx, planes, h, w, ho, wo);
  return vfd::fail_launch("maxpool3s2_bwd");
}

int vfd_normalize_cat(const float* a, const float* b, float* dst, long long n_img, int ca, int cb, int hw,
                      void* stream) {
  VFD_REQUIRE(a && dst && n_img > 0 && ca > 0 && cb >= 0 && (cb == 0 || b) && hw > 0 && hw % 4 == 0 &&
                  (((uintptr_t)a | (uintptr_t)(b ? b : a) | (uintptr_t)dst) & 15) == 0,
              "normalize_cat: bad arguments (hw %% 4 == 0, 16-B aligned)");
  hipStream_t s = (hipStream_t)stream;
  const long long n = n_img * (ca + cb) * (hw / 4);
  vfd::norm_cat_k<<<(unsigned)((n + 255) / 256), 256, 0, s>>>((const float4*)a, (const float4*)(b ? b : a),
                                                              (float4*)dst, n_img, ca, cb, hw / 4);
  return vfd::fail_launch("normalize_cat");
}

int vfd_maxpool3s2_nhwc_fwd(const void* x, void* y, uint8_t* arg, int n, int c, int h, int w, int dtype,
                            void* stream) {
  VFD_REQUIRE(x && y && arg && n > 0 && c > 0 && c % 4 == 0 && h > 0 && w > 0 && (dtype == 0 || dtype == 1) &&
                  (long long)n * h * w * c < (1LL << 31),
              "maxpool3s2_nhwc: bad arguments (C % 4 == 0)");
  hipStream_t s = (hipStream_t)stream;
  vfd::ProfScope ps(vfd::K_MAXPOOL, s);
  const int ho = (h - 1) / 2 + 1, wo = (w - 1) / 2 + 1;
  const long long total = (long long)n * ho * wo * (c / 4);
  const unsigned grid = (unsigned)std::min<long long>((total + 255) / 256, 16384);
  if (dtype == 1)
    vfd::maxpool_nhwc_fwd_k<__bf16><<<grid, 256, 0, s>>>((const __bf16*)x, (__bf16*)y, arg, n, c, h, w, ho, wo);
  else
    vfd::maxpool_nhwc_fwd_k<float><<<grid, 256, 0, s>>>((const float*)x, (float*)y, arg, n, c, h, w, ho, wo);
  return vfd::fail_launch("maxpool3s2_nhwc_fwd");
}

int vfd_maxpool3s2_nhwc_bwd(const void* g, const uint8_t* arg, void* dx, int n, int c, int h, int w, int dtype,
                            void* stream) {
  VFD_REQUIRE(g && arg && dx && n > 0 && c > 0 && c % 4 == 0 && h > 0 && w > 0 && (dtype == 0 || dtype == 1) &&
                  (long long)n * h * w * c < (1LL << 31),
              "maxpool3s2_nhwc: bad arguments (C % 4 == 0)");
  hipStream_t s = (hipStream_t)stream;
  vfd::ProfScope ps(vfd::K_MAXPOOL, s);
  const int ho = (h - 1) / 2 + 1, wo = (w - 1) / 2 + 1;
  const long long total = (long long)n * ((h + 1) / 2) * ((w + 1) / 2) * (c / 4);
  const unsigned grid = (unsigned)std::min<long long>((total + 255) / 256, 16384);
  if (dtype == 1)
    vfd::maxpool_nhwc_bwd_k<__bf16><<<grid, 256, 0, s>>>((const __bf16*)g, arg, (__bf16*)dx, n, c, h, w, ho, wo);
  else
    vfd::maxpool_nhwc_bwd_k<float><<<grid, 256, 0, s>>>((const float*)g, arg, (float*)dx, n, c, h, w, ho, wo);
  return vfd::fail_launch("maxpool3s2_nhwc_bwd");
}

}  // extern "C"
