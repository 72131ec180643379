// Shared helpers of the gfx950 hot-path kernels: error reporting, launch-time profiling hook,
// ATen-compatible sampling arithmetic, wave64 reductions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string>

#include "vfd_capi.h"

namespace vfd {

// ---------------------------------------------------------------- error reporting
void set_error(const char* fmt, ...);
int fail_launch(const char* what);   // reads hipGetLastError, returns VFD_ELAUNCH or VFD_OK

#define VFD_REQUIRE(cond, ...)            \
  do {                                    \
    if (!(cond)) {                        \
      ::vfd::set_error(__VA_ARGS__);      \
      return VFD_EINVAL;                  \
    }                                     \
  } while (0)

// Raise kernel `fn`'s dynamic-LDS limit to `bytes` on the CURRENT device (the attribute is per
// device): set once per (kernel, device), thread-safe (capi.hip).
void lds_attr(const void* fn, int bytes);

// ---------------------------------------------------------------- profiling hook
enum KernelId {
  K_MASK_DOWN = 0, K_FUSE_DEPTH_FWD, K_FUSE_DEPTH_BWD, K_FUSE_POSE_FWD, K_FUSE_POSE_BWD,
  K_VPROJ_FWD, K_VPROJ_BWD, K_VIEW_STATS, K_VIEW_APPLY, K_VIEW_BWD, K_PHOTO_FWD, K_PHOTO_BWD,
  K_SMOOTH_FWD, K_SMOOTH_BWD, K_FUSION_PLAN, K_AGGREGATE, K_VPROJ_PLAN, K_PROJ_CONV_FWD, K_DEPTH_SYN_FWD, K_DEPTH_SYN_BWD, K_PROJ_CONV_DGRAD, K_PAD_CONV_FWD, K_BN_FWD, K_BN_BWD, K_REFLECT_PAD, K_UPSAMPLE_BWD, K_MAXPOOL, K_ELU_PAD, K_DISP_CONV, K_DEC_CONV, K_PROJ_CONV_WGRAD, K_PAD_CONV_DGRAD, K_PAD_CONV_WGRAD, K_LAYOUT_COPY, K_COUNT
};
void prof_begin(int id, hipStream_t s);
void prof_end(int id, hipStream_t s);

struct ProfScope {
  int id;
  hipStream_t s;
  ProfScope(int i, hipStream_t st) : id(i), s(st) { prof_begin(id, s); }
  ~ProfScope() { prof_end(id, s); }
};

// ---------------------------------------------------------------- device math
constexpr int WAVE = 64;

__device__ __forceinline__ float unnorm_ac(float g, int size) {
  // ATen grid_sampler_unnormalize, align_corners=True: ((g + 1) / 2) * (size - 1)
  return ((g + 1.f) / 2.f) * (float)(size - 1);
}

__device__ __forceinline__ int reflect1(int i, int n) {
  // ReflectionPad(1) source index of padded-relative coordinate i in [-1, n]
  return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i);
}

__device__ __forceinline__ bool finitef(float x) { return __builtin_isfinite(x); }

// Stream-K partial sums: s[u] = sum over contributors k (in order) of p_k[u * 64], where p_k =
// partial + contrib[k] * frag + base — U fragment elements of one lane; the loads of two
// contributors x U elements are issued before any add (the reduce kernels are latency-bound), the
// adds keep contributor order (the same sums as a plain loop)
template <int U>
__device__ __forceinline__ void frag_sums(const float* __restrict__ partial, const int* contrib, int nc,
                                          size_t frag, size_t base, float (&s)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) s[u] = 0.f;
  for (int k = 0; k < nc; k += 2) {
    float v0[U], v1[U];
    const float* p0 = partial + (size_t)contrib[k] * frag + base;
    const float* p1 = partial + (size_t)contrib[k + 1 < nc ? k + 1 : k] * frag + base;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v0[u] = p0[u * 64];
      v1[u] = p1[u * 64];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      s[u] += v0[u];
      if (k + 1 < nc) s[u] += v1[u];
    }
  }
}

// Positions of source index i along an axis of length n in a reflect-padded (+1 each side) copy:
// {i+1}, plus 0 when i == 1 and n+1 when i == n-2 (ReflectionPad(1)).  Without padding: {i}.
__device__ __forceinline__ void pad_sets(int i, int n, bool pad, int* idx, int* cnt) {
  if (!pad) { idx[0] = i; *cnt = 1; return; }
  int c = 0;
  idx[c++] = i + 1;
  if (i == 1) idx[c++] = 0;
  if (i == n - 2) idx[c++] = n + 1;
  *cnt = c;
}

// XCD-contiguous workgroup numbering: the hardware deals workgroups round-robin (by linear id) to
// the 8 XCDs, each with its own L2; remapping linear id L to (L % 8) * (total / 8) + L / 8 gives
// each XCD one contiguous run of (x-fastest) tiles, so neighbouring tiles share that XCD's L2.
// Identity when the grid is not a multiple of 8.
__device__ __forceinline__ uint3 xcd_tile() {
  const unsigned total = gridDim.x * gridDim.y * gridDim.z;
  const unsigned L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const unsigned t = (total % 8u == 0u) ? (L % 8u) * (total / 8u) + L / 8u : L;
  return make_uint3(t % gridDim.x, (t / gridDim.x) % gridDim.y, t / (gridDim.x * gridDim.y));
}

// Task index for a 1-D grid of single-task workgroups (grid a multiple of 128): runs of 16
// consecutive tasks go to one XCD (the hardware deals workgroups round-robin to the 8 XCDs), so
// neighbouring tiles share that XCD's L2, while dispatch still follows task order (the split
// tiles' parts, queued first, start first on every XCD).  -1 = beyond the n tasks.
__device__ __forceinline__ int xcd_task(int n) {
  const int k = (int)(blockIdx.x % 8u), j = (int)(blockIdx.x / 8u);
  const int t = ((j / 16) * 8 + k) * 16 + j % 16;
  return t < n ? t : -1;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, WAVE);
  return v;
}

// Bilinear tap set with ATen's corner weights (grid_sampler_2d, zeros padding).
struct Bilinear {
  int x0, y0;
  float w[4];     // nw, ne, sw, se
  bool in[4];
  bool finite;
};

__device__ __forceinline__ Bilinear bilinear_taps(float ix, float iy, int Wd, int Hd) {
  Bilinear b;
  b.finite = finitef(ix) && finitef(iy);
  if (!b.finite) {
    b.x0 = b.y0 = 0;
    for (int k = 0; k < 4; ++k) { b.w[k] = 0.f; b.in[k] = false; }
    return b;
  }
  float fx0 = floorf(ix), fy0 = floorf(iy);
  float fx1 = fx0 + 1.f, fy1 = fy0 + 1.f;
  b.w[0] = (fx1 - ix) * (fy1 - iy);
  b.w[1] = (ix - fx0) * (fy1 - iy);
  b.w[2] = (fx1 - ix) * (iy - fy0);
  b.w[3] = (ix - fx0) * (iy - fy0);
  // clamp before the int conversion: far-away coordinates must not overflow
  fx0 = fminf(fmaxf(fx0, -2.f), (float)Wd + 1.f);
  fy0 = fminf(fmaxf(fy0, -2.f), (float)Hd + 1.f);
  b.x0 = (int)fx0;
  b.y0 = (int)fy0;
  bool xin0 = b.x0 >= 0 && b.x0 < Wd, xin1 = b.x0 + 1 >= 0 && b.x0 + 1 < Wd;
  bool yin0 = b.y0 >= 0 && b.y0 < Hd, yin1 = b.y0 + 1 >= 0 && b.y0 + 1 < Hd;
  b.in[0] = xin0 && yin0;
  b.in[1] = xin1 && yin0;
  b.in[2] = xin0 && yin1;
  b.in[3] = xin1 && yin1;
  return b;
}

// Nearest tap (round half to even, as ATen); returns -1 when out of range / non-finite.
__device__ __forceinline__ int nearest_index(float ix, float iy, int Wd, int Hd) {
  if (!(finitef(ix) && finitef(iy))) return -1;
  float rx = rintf(ix), ry = rintf(iy);
  if (rx < 0.f || rx > (float)(Wd - 1) || ry < 0.f || ry > (float)(Hd - 1)) return -1;
  return (int)ry * Wd + (int)rx;
}

// counter-based normal variates for the identity-loss tie-break noise
__device__ __forceinline__ uint32_t mix32(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)x;
}
__device__ __forceinline__ float hash_normal(uint64_t seed, uint64_t idx) {
  uint32_t a = mix32(seed * 0x9E3779B97F4A7C15ULL + 2 * idx + 1);
  uint32_t b = mix32(seed * 0xD1B54A32D192ED03ULL + 2 * idx + 2);
  float u1 = ((float)(a >> 8) + 1.f) * (1.f / 16777217.f);   // (0, 1]
  float u2 = (float)(b >> 8) * (1.f / 16777216.f);
  return sqrtf(-2.f * logf(u1)) * cosf(6.2831853071795864f * u2);
}

// Sum over a 256-thread block; the total is returned to every thread.  `lds` holds >= 4 T.
template <typename T>
__device__ __forceinline__ T block_sum_all(T v, T* lds) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  return lds[0] + lds[1] + lds[2] + lds[3];
}

// ---------------------------------------------------------------- activation element types
// The dense-net kernels read / write their activations as fp32 or bf16 (config 3's autocast) and
// compute in fp32: loads widen exactly, stores round to nearest even (= torch's .to(bfloat16)).
typedef __bf16 vfd_bf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ float ld1(const __bf16* p) { return (float)*p; }
__device__ __forceinline__ void st1(float* p, float v) { *p = v; }
__device__ __forceinline__ void st1(__bf16* p, float v) { *p = (__bf16)v; }
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 ld4(const __bf16* p) {
  const vfd_bf16x4 v = *reinterpret_cast<const vfd_bf16x4*>(p);
  return make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
}
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ void st4(__bf16* p, float4 v) {
  vfd_bf16x4 b;
  b[0] = (__bf16)v.x;
  b[1] = (__bf16)v.y;
  b[2] = (__bf16)v.z;
  b[3] = (__bf16)v.w;
  *reinterpret_cast<vfd_bf16x4*>(p) = b;
}

// ---------------------------------------------------------------- K3 geometry (frustum samples)
struct Tri {
  int x0, y0, z0;
  float w[8];     // tnw, tne, tsw, tse, bnw, bne, bsw, bse
  unsigned in;
};

// volumetric_fusionnet.py:245-260 + ATen grid_sampler_3d weights
__device__ __forceinline__ Tri frustum_sample(const vfd_voxel_desc& d, const float* __restrict__ iK,
                                              const float* __restrict__ E, int px, int py, float dep) {
  float fx = (float)px, fy = (float)py;
  float r0 = iK[0] * fx + iK[1] * fy + iK[2];
  float r1 = iK[4] * fx + iK[5] * fy + iK[6];
  float r2 = iK[8] * fx + iK[9] * fy + iK[10];
  float p0 = dep * r0, p1 = dep * r1, p2 = dep * r2;
  float w0 = E[0] * p0 + E[1] * p1 + E[2] * p2 + E[3];
  float w1 = E[4] * p0 + E[5] * p1 + E[6] * p2 + E[7];
  float w2 = E[8] * p0 + E[9] * p1 + E[10] * p2 + E[11];
  float gx = (w0 - d.str[0]) / d.len[0] * 2.f - 1.f;
  float gy = (w1 - d.str[1]) / d.len[1] * 2.f - 1.f;
  float gz = (w2 - d.str[2]) / d.len[2] * 2.f - 1.f;
  float ix = unnorm_ac(gx, d.X), iy = unnorm_ac(gy, d.Y), iz = unnorm_ac(gz, d.Z);
  Tri t;
  t.in = 0;
  if (!(finitef(ix) && finitef(iy) && finitef(iz))) {
    t.x0 = t.y0 = t.z0 = -4;
    for (int k = 0; k < 8; ++k) t.w[k] = 0.f;
    return t;
  }
  float fx0 = floorf(ix), fy0 = floorf(iy), fz0 = floorf(iz);
  float fx1 = fx0 + 1.f, fy1 = fy0 + 1.f, fz1 = fz0 + 1.f;
  float ax[2] = {fx1 - ix, ix - fx0}, ay[2] = {fy1 - iy, iy - fy0}, az[2] = {fz1 - iz, iz - fz0};
  t.x0 = (int)fminf(fmaxf(fx0, -4.f), (float)d.X + 4.f);
  t.y0 = (int)fminf(fmaxf(fy0, -4.f), (float)d.Y + 4.f);
  t.z0 = (int)fminf(fmaxf(fz0, -4.f), (float)d.Z + 4.f);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    int dx = k & 1, dy = (k >> 1) & 1, dz = k >> 2;
    int xx = t.x0 + dx, yy = t.y0 + dy, zz = t.z0 + dz;
    bool ok = xx >= 0 && xx < d.X && yy >= 0 && yy < d.Y && zz >= 0 && zz < d.Z;
    t.w[k] = ax[dx] * ay[dy] * az[dz];
    t.in |= (ok ? 1u : 0u) << k;
  }
  return t;
}

__device__ __forceinline__ int tri_index(const vfd_voxel_desc& d, const Tri& t, int k) {
  return ((t.z0 + (k >> 2)) * d.Y + (t.y0 + ((k >> 1) & 1))) * d.X + (t.x0 + (k & 1));
}

__device__ __forceinline__ int corner_offset(const vfd_voxel_desc& d, int k) {
  return (k & 1) + ((k >> 1) & 1) * d.X + (k >> 2) * d.X * d.Y;
}

__host__ __device__ inline unsigned cdiv(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

// Zero fill as a kernel (instead of hipMemsetAsync): a plain kernel node when a step is captured into
// a HIP graph, 16-B stores, byte tail.  Zeroed counters / accumulators ahead of atomics use it.
template <int Unused = 0>
__global__ __launch_bounds__(256) void zero_fill_k(unsigned char* __restrict__ p, size_t bytes) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t mis = (size_t)((16u - ((uintptr_t)p & 15u)) & 15u);
  const size_t head = mis < bytes ? mis : bytes;            // bytes up to the first 16-B boundary
  unsigned char* q = p + head;
  const size_t n16 = (bytes - head) / 16, tail = bytes - head - n16 * 16;
  if (i < head) p[i] = 0;
  for (size_t k = i; k < n16; k += stride) reinterpret_cast<uint4*>(q)[k] = make_uint4(0u, 0u, 0u, 0u);
  if (i < tail) q[n16 * 16 + i] = 0;
}

static inline void zero_async(void* p, size_t bytes, hipStream_t s) {
  if (bytes == 0) return;
  size_t blocks = (bytes / 16 + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks);
  zero_fill_k<<<(unsigned)blocks, 256, 0, s>>>((unsigned char*)p, bytes);
}

}  // namespace vfd
