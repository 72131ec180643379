// MaxPool2d(3, stride 2, padding 1) of the ResNet stem (torchvision / packnet ResnetEncoder,
// fusion_depthnet.py:24-36, fusion_posenet.py:22-35), NCHW fp32, forward and backward.
// The forward keeps the winning window position as one byte (ATen stores an int64 index: 8x the
// bytes); ties go to the first maximum in window scan order and NaN wins, as ATen's `val > max ||
// isnan(val)` does.  The backward is a gather: every input pixel sums the gradients of the (<= 4)
// output windows whose winner it is, in a fixed order (deterministic, no atomics).
#include "vfd_common.h"

namespace vfd {

__global__ __launch_bounds__(256) void maxpool_fwd_k(const float* __restrict__ x, float* __restrict__ y,
                                                     uint8_t* __restrict__ arg, long long planes, int h, int w,
                                                     int ho, int wo) {
  // grid (cdiv(ho*wo, 256), planes): 32-bit index math inside a plane (64-bit division is a
  // long software sequence on CDNA and made this kernel ALU-bound)
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ho * wo) return;
  const int oy = j / wo, ox = j - oy * wo;
  for (long long p = blockIdx.y; p < planes; p += gridDim.y) {
    const size_t i = (size_t)p * ho * wo + j;
    const float* xp = x + (size_t)p * h * w;
    float best = -INFINITY;
    int bi = 4;                                      // centre (always inside the image)
    bool first = true;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int yy = 2 * oy - 1 + ky;
      if (yy < 0 || yy >= h) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int xx = 2 * ox - 1 + kx;
        if (xx < 0 || xx >= w) continue;
        const float v = xp[yy * w + xx];
        if (first || v > best || isnan(v)) {
          best = v;
          bi = ky * 3 + kx;
          first = false;
        }
      }
    }
    y[i] = best;
    arg[i] = (uint8_t)bi;
  }
}

__global__ __launch_bounds__(256) void maxpool_bwd_k(const float* __restrict__ g, const uint8_t* __restrict__ arg,
                                                     float* __restrict__ dx, long long planes, int h, int w, int ho,
                                                     int wo) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= h * w) return;
  const int yy = j / w, xx = j - yy * w;
  // output rows / columns whose window (2o-1 .. 2o+1) contains the pixel, in increasing order:
  // o in {p/2, p/2 + 1} (the second only for odd p)
  const int oy0 = yy / 2, ox0 = xx / 2;
  const bool y2 = (yy & 1) && oy0 + 1 < ho, x2 = (xx & 1) && ox0 + 1 < wo;
  const int o00 = oy0 * wo + ox0;
  const int k00 = (yy - 2 * oy0 + 1) * 3 + (xx - 2 * ox0 + 1);   // window position in (oy0, ox0)
  for (long long p = blockIdx.y; p < planes; p += gridDim.y) {
    const float* gp = g + (size_t)p * ho * wo;
    const uint8_t* ap = arg + (size_t)p * ho * wo;
    float acc = 0.f;
    if (ap[o00] == k00) acc += gp[o00];
    if (x2 && ap[o00 + 1] == k00 - 2) acc += gp[o00 + 1];
    if (y2 && ap[o00 + wo] == k00 - 6) acc += gp[o00 + wo];
    if (y2 && x2 && ap[o00 + wo + 1] == k00 - 8) acc += gp[o00 + wo + 1];
    dx[(size_t)p * h * w + j] = acc;
  }
}

}  // namespace vfd

extern "C" {

int vfd_maxpool3s2_fwd(const float* x, float* y, uint8_t* arg, long long planes, int h, int w, void* stream) {
  VFD_REQUIRE(x && y && arg && planes > 0 && h > 0 && w > 0 && (long long)h * w < (1LL << 31),
              "maxpool3s2: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  vfd::ProfScope ps(vfd::K_MAXPOOL, s);
  const int ho = (h - 1) / 2 + 1, wo = (w - 1) / 2 + 1;
  const unsigned gy = (unsigned)(planes < 65535 ? planes : 65535);
  vfd::maxpool_fwd_k<<<dim3((unsigned)((ho * wo + 255) / 256), gy), 256, 0, s>>>(x, y, arg, planes, h, w, ho, wo);
  return vfd::fail_launch("maxpool3s2_fwd");
}

int vfd_maxpool3s2_bwd(const float* g, const uint8_t* arg, float* dx, long long planes, int h, int w, void* stream) {
  VFD_REQUIRE(g && arg && dx && planes > 0 && h > 0 && w > 0 && (long long)h * w < (1LL << 31),
              "maxpool3s2: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  vfd::ProfScope ps(vfd::K_MAXPOOL, s);
  const int ho = (h - 1) / 2 + 1, wo = (w - 1) / 2 + 1;
  const unsigned gy = (unsigned)(planes < 65535 ? planes : 65535);
  vfd::maxpool_bwd_k<<<dim3((unsigned)((h * w + 255) / 256), gy), 256, 0, s>>>(g, arg, dx, planes, h, w, ho, wo);
  return vfd::fail_launch("maxpool3s2_bwd");
}

}  // extern "C"
