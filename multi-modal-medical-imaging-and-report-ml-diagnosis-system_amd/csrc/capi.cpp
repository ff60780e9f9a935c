// C-ABI plumbing: version + thread-local error message.
#include <stdarg.h>
#include <stdio.h>

#include "../../include/mmdx.h"

static thread_local char g_err[512] = "";

extern "C" void mmdx_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* mmdx_last_error(void) { return g_err; }

extern "C" int mmdx_version(void) { return 1; }
