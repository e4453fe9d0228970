// Error reporting and version for the libtmr C ABI.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"
#include "tmr.h"

static thread_local char g_err[1024] = "";

void tmr_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

TMR_API const char* tmr_last_error(void) { return g_err; }
TMR_API void tmr_clear_error(void) { g_err[0] = 0; }
TMR_API int tmr_abi_version(void) { return TMR_ABI_VERSION; }
