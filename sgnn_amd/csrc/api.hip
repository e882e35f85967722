// Host-side status / error plumbing of the C-ABI (include/sgnn.h).
#include <stdio.h>
#include <string.h>

#include "sgnn_internal.h"

namespace {
thread_local char g_err[512] = "";
}

namespace sgnn {

int set_error(int status, const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return status;
}

int check_launch(const char* where) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "%s: %s", where, hipGetErrorString(e));
    return SGNN_ERR_HIP;
  }
  return SGNN_OK;
}

}  // namespace sgnn

extern "C" const char* sgnn_version(void) { return "sgnn-mi355x 0.6 (abi 6, gfx950, fp32 MFMA)"; }
extern "C" int32_t sgnn_abi_version(void) { return SGNN_ABI_VERSION; }
extern "C" int32_t sgnn_step_flag_words(void) { return SGNN_STEP_FLAG_WORDS; }
extern "C" const char* sgnn_last_error(void) { return g_err; }
