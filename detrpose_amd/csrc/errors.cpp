// Thread-local error string behind dp_last_error() (include/detrpose_hip.h).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/detrpose_hip.h"

static thread_local char g_err[512] = "";

void dp_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int dp_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    dp_set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

static thread_local char* g_describe = nullptr;
static thread_local int g_describe_len = 0;
char* dp_describe_buf(int* len) {
  *len = g_describe_len;
  return g_describe;
}
void dp_describe_set(char* buf, int len) {
  g_describe = buf;
  g_describe_len = len;
}

extern "C" const char* dp_last_error(void) { return g_err; }
extern "C" int dp_version(void) { return 1; }
