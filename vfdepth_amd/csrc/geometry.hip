// Batched general 4x4 inverse (the extrinsics' inverse of estimate_vfdepth, models/vfdepth.py:211,
// and the depth-synthesis transforms): one thread per matrix, by cofactors in exactly the operation
// order of geometry.inverse4x4 (its torch restatement), so the two agree bit for bit (fp-contract
// off).  It replaces ~150 single-element ATen launches per step; capturable (no solver, no sync).
#include "vfd_common.h"

namespace vfd {

__global__ __launch_bounds__(64) void inverse4x4_k(const float* __restrict__ m, float* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* a = m + (size_t)i * 16;
  const float a00 = a[0], a01 = a[1], a02 = a[2], a03 = a[3];
  const float a10 = a[4], a11 = a[5], a12 = a[6], a13 = a[7];
  const float a20 = a[8], a21 = a[9], a22 = a[10], a23 = a[11];
  const float a30 = a[12], a31 = a[13], a32 = a[14], a33 = a[15];
  const float s0 = a00 * a11 - a10 * a01, s1 = a00 * a12 - a10 * a02, s2 = a00 * a13 - a10 * a03;
  const float s3 = a01 * a12 - a11 * a02, s4 = a01 * a13 - a11 * a03, s5 = a02 * a13 - a12 * a03;
  const float c5 = a22 * a33 - a32 * a23, c4 = a21 * a33 - a31 * a23, c3 = a21 * a32 - a31 * a22;
  const float c2 = a20 * a33 - a30 * a23, c1 = a20 * a32 - a30 * a22, c0 = a20 * a31 - a30 * a21;
  const float det = s0 * c5 - s1 * c4 + s2 * c3 + s3 * c2 - s4 * c1 + s5 * c0;
  float v[16];
  v[0] = a11 * c5 - a12 * c4 + a13 * c3;
  v[1] = -a01 * c5 + a02 * c4 - a03 * c3;
  v[2] = a31 * s5 - a32 * s4 + a33 * s3;
  v[3] = -a21 * s5 + a22 * s4 - a23 * s3;
  v[4] = -a10 * c5 + a12 * c2 - a13 * c1;
  v[5] = a00 * c5 - a02 * c2 + a03 * c1;
  v[6] = -a30 * s5 + a32 * s2 - a33 * s1;
  v[7] = a20 * s5 - a22 * s2 + a23 * s1;
  v[8] = a10 * c4 - a11 * c2 + a13 * c0;
  v[9] = -a00 * c4 + a01 * c2 - a03 * c0;
  v[10] = a30 * s4 - a31 * s2 + a33 * s0;
  v[11] = -a20 * s4 + a21 * s2 - a23 * s0;
  v[12] = -a10 * c3 + a11 * c1 - a12 * c0;
  v[13] = a00 * c3 - a01 * c1 + a02 * c0;
  v[14] = -a30 * s3 + a31 * s1 - a32 * s0;
  v[15] = a20 * s3 - a21 * s1 + a22 * s0;
  float* o = out + (size_t)i * 16;
#pragma unroll
  for (int k = 0; k < 16; ++k) o[k] = v[k] / det;
}

}  // namespace vfd

extern "C" int vfd_inverse4x4(const float* m, float* out, int n, void* stream) {
  VFD_REQUIRE(m && out && n > 0, "inverse4x4: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  vfd::inverse4x4_k<<<(n + 63) / 64, 64, 0, s>>>(m, out, n);
  return vfd::fail_launch("inverse4x4");
}
