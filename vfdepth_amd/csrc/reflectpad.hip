// Reflect padding by one pixel (nn.Conv2d(padding_mode='reflect', padding=1): the decoders'
// 3x3 convs, network/blocks.py conv2d blocks) for NCHW fp32 maps, forward and backward.
// The backward is a gather: every input pixel sums its (up to four) padded copies in a fixed
// order (pad_sets), so it needs no atomics and is deterministic (ATen's reflection_pad2d
// backward scatters with atomics).
#include "vfd_common.h"

namespace vfd {

__device__ __forceinline__ int rp_src(int i, int n) {       // padded index -> source index
  return i == 0 ? 1 : (i == n + 1 ? n - 2 : i - 1);
}

__global__ __launch_bounds__(256) void reflect_pad_fwd_k(const float* __restrict__ x, float* __restrict__ y,
                                                         long long planes, int h, int w) {
  const int ho = h + 2, wo = w + 2;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;       // pixel of the padded plane
  if (j >= ho * wo) return;
  const int Y = j / wo, X = j - Y * wo;
  const int src = rp_src(Y, h) * w + rp_src(X, w);
  for (long long p = blockIdx.y; p < planes; p += gridDim.y) y[p * ho * wo + j] = x[p * h * w + src];
}

__global__ __launch_bounds__(256) void reflect_pad_bwd_k(const float* __restrict__ g, float* __restrict__ dx,
                                                         long long planes, int h, int w) {
  const int wo = w + 2;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;       // pixel of the plane
  if (j >= h * w) return;
  const int yy = j / w, x = j - yy * w;
  int rows[3], cols[3], nr, nc;
  pad_sets(yy, h, true, rows, &nr);
  pad_sets(x, w, true, cols, &nc);
  for (long long p = blockIdx.y; p < planes; p += gridDim.y) {
    const float* gp = g + p * (h + 2) * wo;
    float s = 0.f;
    for (int a = 0; a < nr; ++a)
      for (int b = 0; b < nc; ++b) s += gp[rows[a] * wo + cols[b]];
    dx[p * h * w + j] = s;
  }
}

// Backward of LeakyReLU(slope) followed by the one-pixel reflect pad, channels-last (the fused
// reduce_dim convs' outputs, projconv.hip / padconv.hip): gp[n][y][x][c] = (sum of the copies of
// g at pixel (y, x)) * (out[n][y+1][x+1][c] > 0 ? 1 : slope); float4 lanes over channels.
__global__ __launch_bounds__(256) void lrelu_pad_bwd_nhwc_k(const float4* __restrict__ g, const float4* __restrict__ out,
                                                            float4* __restrict__ gp, long long n_img, int h, int w,
                                                            int c4, float slope) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;       // (pixel, float4) of image blockIdx.y
  if (j >= h * w * c4) return;
  const long long n = blockIdx.y;
  const int pix = j / c4, q = j - pix * c4;
  const int yy = pix / w, x = pix - yy * w;
  const int wo = w + 2;
  const size_t i = (size_t)n * h * w * c4 + j;
  int rows[3], cols[3], nr, nc;
  pad_sets(yy, h, true, rows, &nr);
  pad_sets(x, w, true, cols, &nc);
  const float4* gb = g + n * (h + 2) * wo * c4 + q;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int a = 0; a < nr; ++a)
    for (int b = 0; b < nc; ++b) {
      const float4 v = gb[((size_t)rows[a] * wo + cols[b]) * c4];
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
  const float4 o = out[((n * (h + 2) + yy + 1) * wo + x + 1) * c4 + q];
  s.x *= o.x > 0.f ? 1.f : slope;
  s.y *= o.y > 0.f ? 1.f : slope;
  s.z *= o.z > 0.f ? 1.f : slope;
  s.w *= o.w > 0.f ? 1.f : slope;
  gp[i] = s;
}

}  // namespace vfd

using namespace vfd;

extern "C" {

int vfd_reflect_pad1_fwd(const float* x, float* y, long long planes, int h, int w, void* stream) {
  VFD_REQUIRE(x && y && planes > 0 && h >= 2 && w >= 2 && (long long)(h + 2) * (w + 2) < (1LL << 31),
              "reflect_pad1: bad arguments (h, w >= 2)");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_REFLECT_PAD, s);
  const dim3 grid((unsigned)(((h + 2) * (w + 2) + 255) / 256), (unsigned)(planes < 65535 ? planes : 65535));
  reflect_pad_fwd_k<<<grid, 256, 0, s>>>(x, y, planes, h, w);
  return fail_launch("reflect_pad1_fwd");
}

int vfd_reflect_pad1_bwd(const float* g, float* dx, long long planes, int h, int w, void* stream) {
  VFD_REQUIRE(g && dx && planes > 0 && h >= 2 && w >= 2 && (long long)(h + 2) * (w + 2) < (1LL << 31),
              "reflect_pad1: bad arguments (h, w >= 2)");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps(K_REFLECT_PAD, s);
  const dim3 grid((unsigned)((h * w + 255) / 256), (unsigned)(planes < 65535 ? planes : 65535));
  reflect_pad_bwd_k<<<grid, 256, 0, s>>>(g, dx, planes, h, w);
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
  lrelu_pad_bwd_nhwc_k<<<grid, 256, 0, s>>>((const float4*)g, (const float4*)out, (float4*)gp,
                                                                  n_img, h, w, C / 4, slope);
  return fail_launch("lrelu_pad1_bwd_nhwc");
}

}  // extern "C"
