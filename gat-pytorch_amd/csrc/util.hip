// Error reporting and version of libgatx.so (C-ABI, include/gatx.h).
#include <stdarg.h>

#include "gatx_common.h"

namespace gatx {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace gatx

extern "C" const char* gatx_last_error(void) { return gatx::g_err; }
extern "C" int gatx_version(void) { return 1; }
