// Thread-local error message + ABI version for libic2ops.
#include "common.h"

#include <cstdio>
#include <cstdlib>

namespace ic2 {
static thread_local char g_err[1024] = "no error";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// Development knobs (A/B switches and forced kernel instances for the tests): the library's launch plan depends on
// the process environment ONLY when IC2_DEV=1 is set; otherwise every knob returns its default.
int knob(const char* name, int dflt) {
  static const bool dev = [] {
    const char* e = getenv("IC2_DEV");
    return e && e[0] == '1';
  }();
  const char* e = getenv(name);
  if (!dev) {
    // a knob set without IC2_DEV=1 is ignored: say so once per knob (an A/B script would otherwise compare default
    // against default)
    if (e) fprintf(stderr, "[ic2] %s=%s ignored: development knobs need IC2_DEV=1\n", name, e);
    return dflt;
  }
  return e ? atoi(e) : dflt;
}
}  // namespace ic2

extern "C" int ic2_dev_mode(void) {
  const char* e = getenv("IC2_DEV");
  return e && e[0] == '1';
}
extern "C" const char* ic2_last_error(void) { return ic2::g_err; }
extern "C" int ic2_abi_version(void) { return 1; }
