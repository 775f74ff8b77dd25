// ABI bookkeeping: version and thread-local error text.
#include "common.h"

#include <cstring>

namespace ewvit {
static thread_local char g_err[512] = "";
// per host thread: nn.DataParallel runs its replicas in threads (reference train.py:249-251),
// and a cap set around one replica's branch must not reach another's launches
thread_local int g_grid_cap = 0;

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace ewvit

extern "C" int ewvit_abi_version(void) { return EWVIT_ABI_VERSION; }
extern "C" const char *ewvit_last_error(void) { return ewvit::g_err; }

// workgroups at most per launch of the big-grid kernels (LDS-DMA convs, BatchNorm passes);
// 0 = no cap.  Set around a branch that shares the GPU with another stream; the cap is the
// calling thread's (launches issued by other threads keep their own).
extern "C" int ewvit_set_grid_cap(int max_workgroups) {
  const int prev = ewvit::g_grid_cap;
  ewvit::g_grid_cap = max_workgroups > 0 ? (max_workgroups + 7) / 8 * 8 : 0;   // whole XCD rounds
  return prev;
}

using namespace ewvit;

// Timeline probe (diagnostics, tools/step_timeline.py): when the stream reaches it, one lane
// writes the device wall clock (ewvit_wall_clock_khz ticks per millisecond) to stamps[idx].
__global__ void probe_kernel(long long *stamps, int idx) {
  const int t = (int)threadIdx.x;
  if (t == 0) stamps[idx + t] = wall_clock64();
}

extern "C" int ewvit_probe(long long *stamps, int idx, void *stream) {
  EWVIT_CHECK_ARG(stamps && idx >= 0, "probe: bad args");
  hipLaunchKernelGGL(probe_kernel, dim3(1), dim3(64), 0, as_stream(stream), stamps, idx);
  return launch_status("probe");
}

extern "C" int ewvit_wall_clock_khz(void) {
  int dev = 0, v = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, dev) != hipSuccess)
    return 0;
  return v;
}
