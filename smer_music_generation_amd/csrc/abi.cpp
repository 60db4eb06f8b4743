// Status / version entries of the C-ABI.
#include <hip/hip_runtime.h>
#include <string.h>

#include "../../include/smer_hip.h"

static thread_local char g_err[512] = "";

extern "C" int smer_set_error(int code, const char* msg) {
  strncpy(g_err, msg ? msg : "", sizeof(g_err) - 1);
  g_err[sizeof(g_err) - 1] = 0;
  return code;
}
extern "C" const char* smer_last_error(void) { return g_err; }
extern "C" int smer_abi_version(void) { return 1; }
