// C-ABI plumbing: version, thread-local error string, and the launch-time profiling hook that
// bench.py uses to time one kernel with HIP events on the stream it is launched on.
#include <stdarg.h>

#include <mutex>
#include <set>
#include <utility>
#include <vector>

#include "vfd_common.h"

namespace vfd {

static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

int fail_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return VFD_ELAUNCH;
  }
  return VFD_OK;
}

void lds_attr(const void* fn, int bytes) {
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> done;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(mu);
  if (done.insert({fn, dev}).second)
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// ---------------------------------------------------------------- profiling
struct Prof {
  std::mutex mu;
  int kernel = -2;                  // -2: off, -1: every kernel, >= 0: one kernel
  std::vector<hipEvent_t> pool;     // [start, end] pairs
  std::vector<int> ids;             // kernel id of each pair
  size_t used = 0;
};
static Prof g_prof;

static hipEvent_t prof_event() {
  if (g_prof.used == g_prof.pool.size()) {
    hipEvent_t e;
    (void)hipEventCreate(&e);
    g_prof.pool.push_back(e);
  }
  return g_prof.pool[g_prof.used++];
}

static bool prof_on(int id) { return g_prof.kernel == -1 || (g_prof.kernel >= 0 && id == g_prof.kernel); }

void prof_begin(int id, hipStream_t s) {
  if (!prof_on(id)) return;
  std::lock_guard<std::mutex> lk(g_prof.mu);
  const size_t pair = g_prof.used / 2;
  if (g_prof.ids.size() <= pair) g_prof.ids.resize(pair + 1);
  g_prof.ids[pair] = id;
  (void)hipEventRecord(prof_event(), s);
}

void prof_end(int id, hipStream_t s) {
  if (!prof_on(id)) return;
  std::lock_guard<std::mutex> lk(g_prof.mu);
  (void)hipEventRecord(prof_event(), s);
}

static const char* kNames[K_COUNT] = {
  "mask_downsample", "fuse_depth_fwd", "fuse_depth_bwd", "fuse_pose_fwd", "fuse_pose_bwd",
  "voxel_project_fwd", "voxel_project_bwd", "view_stats", "view_apply", "view_bwd",
  "photo_fwd", "photo_bwd", "smooth_fwd", "smooth_bwd", "fusion_plan", "aggregate", "voxel_project_plan",
  "proj_conv_fwd", "depth_syn_fwd", "depth_syn_bwd", "proj_conv_dgrad", "pad_conv_fwd", "bn_fwd", "bn_bwd", "reflect_pad", "upsample_bwd", "maxpool", "elu_pad", "disp_conv", "dec_conv", "proj_conv_wgrad", "pad_conv_dgrad", "pad_conv_wgrad", "layout_copy"};

}  // namespace vfd

extern "C" {

int vfd_version(void) { return 1; }

const char* vfd_last_error(void) { return vfd::g_err.c_str(); }

const char* vfd_kernel_name(int id) { return (id >= 0 && id < vfd::K_COUNT) ? vfd::kNames[id] : ""; }

int vfd_prof_enable(int id) {
  std::lock_guard<std::mutex> lk(vfd::g_prof.mu);
  vfd::g_prof.kernel = id;
  vfd::g_prof.used = 0;
  return VFD_OK;
}

int vfd_prof_read(int* launches, double* total_ms) {
  return vfd_prof_read_kernels(VFD_PROF_ALL, launches, total_ms);
}

int vfd_prof_read_kernels(int count, int* launches, double* total_ms) {
  // per-kernel launches / summed milliseconds of every recorded pair; resets the record.
  // count == VFD_PROF_ALL: one aggregate value in launches[0] / total_ms[0].
  std::lock_guard<std::mutex> lk(vfd::g_prof.mu);
  const int n_out = count == VFD_PROF_ALL ? 1 : count;
  for (int k = 0; k < n_out; ++k) {
    if (launches) launches[k] = 0;
    if (total_ms) total_ms[k] = 0.0;
  }
  for (size_t i = 0; i + 1 < vfd::g_prof.used; i += 2) {
    (void)hipEventSynchronize(vfd::g_prof.pool[i + 1]);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, vfd::g_prof.pool[i], vfd::g_prof.pool[i + 1]) != hipSuccess) continue;
    const int id = count == VFD_PROF_ALL ? 0 : vfd::g_prof.ids[i / 2];
    if (id < 0 || id >= n_out) continue;
    if (launches) launches[id] += 1;
    if (total_ms) total_ms[id] += ms;
  }
  vfd::g_prof.used = 0;
  return VFD_OK;
}

}  // extern "C"
