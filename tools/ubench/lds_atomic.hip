// Micro-benchmark: LDS float RMW forms on gfx950 — ds_add_f32 (atomic) vs read+add+write, lanes
// on consecutive addresses (no conflicts) and all lanes on one address.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
  __shared__ float t[64 * 64];
  for (int i = threadIdx.x; i < 64 * 64; i += 256) t[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float v = 1.0f + lane;
  for (int it = 0; it < iters; ++it) {
    const int row = (it * 7 + wv * 13) & 63;
    if (MODE == 0) atomicAdd(&t[row * 64 + lane], v);                 // ds_add_f32, distinct addresses
    else if (MODE == 1) t[(wv * 16 + (it & 15)) * 64 + lane] += v;    // private rows: read + add + write
    else if (MODE == 2) atomicAdd(&t[row * 64], v);                   // all lanes one address
    else if (MODE == 3) __hip_atomic_fetch_add(&t[row * 64 + lane], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  float s = 0.f;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) s += t[i];
  if (s == 12345.f) out[0] = s;
}

template <int MODE>
float run(float* out, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  k<MODE><<<1024, 256>>>(out, iters);
  hipEventRecord(a);
  k<MODE><<<1024, 256>>>(out, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  float* out; hipMalloc(&out, 4);
  const int iters = 4096;
  const double ops = 1024.0 * 4 * iters;   // wave-instructions
  const char* names[] = {"ds_add_f32 distinct", "read+add+write private", "ds_add_f32 one address", "atomic relaxed wg distinct"};
  float t0 = run<0>(out, iters), t1 = run<1>(out, iters), t2 = run<2>(out, iters), t3 = run<3>(out, iters);
  float ts[] = {t0, t1, t2, t3};
  for (int m = 0; m < 4; ++m)
    printf("%-28s %8.3f ms  %6.2f ns/wave-op/CU  (%.1f cycles @2.4GHz per wave-op per CU)\n", names[m], ts[m],
           ts[m] * 1e6 / (ops / 256), ts[m] * 1e6 / (ops / 256) * 2.4);
  return 0;
}
