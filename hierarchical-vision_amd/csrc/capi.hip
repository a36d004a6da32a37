// C-ABI status plumbing for libhvk: error codes + last-error text (thread-local).
#include <stdarg.h>
#include <stdio.h>

#include "hvk_common.h"

static thread_local char g_hvk_err[512] = "";

extern "C" {

int hvk_set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_hvk_err, sizeof(g_hvk_err), fmt, ap);
  va_end(ap);
  return code;
}

const char* hvk_last_error_string(void) { return g_hvk_err; }

int hvk_abi_version(void) { return 1; }

}  // extern "C"
