// Thread-local error message + ABI version for libic2ops.
#include "common.h"

namespace ic2 {
static thread_local char g_err[1024] = "no error";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace ic2

extern "C" const char* ic2_last_error(void) { return ic2::g_err; }
extern "C" int ic2_abi_version(void) { return 1; }
