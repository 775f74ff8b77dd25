// ABI bookkeeping: version and thread-local error text.
#include "common.h"

#include <cstring>

namespace ewvit {
static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace ewvit

extern "C" int ewvit_abi_version(void) { return EWVIT_ABI_VERSION; }
extern "C" const char *ewvit_last_error(void) { return ewvit::g_err; }
