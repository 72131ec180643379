// Known-byte probes for rocprofv3's FETCH_SIZE on gfx950 (MI355X_MICROARCH.md: FETCH_SIZE reports
// half the bytes of 16-B-per-lane streaming reads): each kernel reads an n-float buffer exactly
// once with 4-, 8- or 16-B lanes (fully coalesced, grid-stride) and writes one float per block.
#include <hip/hip_runtime.h>

template <typename T>
__global__ __launch_bounds__(256) void probe_read_k(const T* __restrict__ src, size_t n, float* __restrict__ out) {
  float acc = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const T v = src[i];
    const float* f = reinterpret_cast<const float*>(&v);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k) acc += f[k];
  }
  __shared__ float s[256];
  s[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < 256; ++i) t += s[i];
    out[blockIdx.x] = t;
  }
}

extern "C" int probe_read(const float* src, size_t nfloat, int width, float* out, int blocks, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (width == 4) probe_read_k<float><<<blocks, 256, 0, s>>>(src, nfloat, out);
  else if (width == 8) probe_read_k<float2><<<blocks, 256, 0, s>>>((const float2*)src, nfloat / 2, out);
  else probe_read_k<float4><<<blocks, 256, 0, s>>>((const float4*)src, nfloat / 4, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
