// C-ABI plumbing: version + thread-local error message.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include <mutex>
#include <vector>

#include <hip/hip_ext.h>

#include "../../include/mmdx.h"
#include "common.h"

static thread_local char g_err[512] = "";

extern "C" void mmdx_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* mmdx_last_error(void) { return g_err; }

extern "C" int mmdx_version(void) { return 1; }

namespace mmdx {

static long env_long(const char* name, long dflt) {
  const char* e = getenv(name);
  return e && *e ? atol(e) : dflt;
}

static Knobs read_knobs() {
  Knobs k;
  const long w = env_long("MMDX_CONV_N64_WIDE", -1);
  k.conv_n64_wide = w < 0 ? -1 : w == 0 ? 0 : 1;
  k.conv_8w128 = env_long("MMDX_CONV_8W128", 1) != 0;
  k.stem_direct = env_long("MMDX_STEM_DIRECT", 1) != 0;
  const long t = env_long("MMDX_WGRAD_TARGET", 256);
  k.wgrad_target = t >= 64 && t <= 4096 ? t : 256;
  k.wgrad_rq = env_long("MMDX_WGRAD_RQ", 1) != 0;
  k.gemm256_fwd_min = env_long("MMDX_GEMM256_FWD_MIN", 90);
  k.gemm_8w128 = env_long("MMDX_GEMM_8W128", 1) != 0;
  const long s = env_long("MMDX_SPLITK_TARGET", 256);
  k.splitk_target = s >= 64 ? s : 256;
  k.splitk_vec = env_long("MMDX_SPLITK_VEC", 1) != 0;
  k.wgrad_bias_fused = env_long("MMDX_WGRAD_BIAS_FUSED", 1) != 0;
  k.bias_grad_gemm = env_long("MMDX_BIAS_GRAD_GEMM", 0) == 1;
  k.ln_bwd_rpw = env_long("MMDX_LN_BWD_RPW", 8) == 4 ? 4 : 8;
  k.attn_fwd_nw = (int)env_long("MMDX_ATTN_FWD_NW", 0);
  k.attn_bwd_nw = (int)env_long("MMDX_ATTN_BWD_NW", 0);
  k.lstm_bwd_probe = env_long("MMDX_LSTM_BWD_PROBE", 0) != 0;
  return k;
}

static Knobs g_knobs;
static std::once_flag g_knobs_once;

const Knobs& knobs() {
  std::call_once(g_knobs_once, [] { g_knobs = read_knobs(); });
  return g_knobs;
}

}  // namespace mmdx

extern "C" int mmdx_reload_config(void) {
  mmdx::knobs();  // the first read, if it has not happened yet
  mmdx::g_knobs = mmdx::read_knobs();
  return 0;
}

// A HIP stream restricted to `cus` of the device's compute units (0 or >= the device's
// count: all of them), spread evenly over the mask so every XCD keeps its share; priority as
// hipStreamCreateWithPriority.  The caller owns it (mmdx_stream_destroy).
extern "C" int mmdx_stream_create(int priority, int cus, void** out) {
  MMDX_CHECK_ARG(out, "mmdx_stream_create: out is NULL");
  *out = nullptr;
  int dev = 0, n = 0;
  MMDX_CHECK_ARG(hipGetDevice(&dev) == hipSuccess &&
                     hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) ==
                         hipSuccess && n > 0,
                 "mmdx_stream_create: no device");
  hipStream_t s = nullptr;
  if (cus <= 0 || cus >= n) {
    MMDX_CHECK_ARG(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority) == hipSuccess,
                   "mmdx_stream_create: hipStreamCreateWithPriority failed");
  } else {
    std::vector<uint32_t> mask((n + 31) / 32, 0u);
    for (int i = 0; i < cus; ++i) {
      const int cu = (int)((long)i * n / cus);  // evenly spaced
      mask[cu / 32] |= 1u << (cu % 32);
    }
    MMDX_CHECK_ARG(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) ==
                       hipSuccess,
                   "mmdx_stream_create: hipExtStreamCreateWithCUMask failed");
  }
  *out = (void*)s;
  return 0;
}

extern "C" int mmdx_stream_destroy(void* s) {
  MMDX_CHECK_ARG(s && hipStreamDestroy((hipStream_t)s) == hipSuccess, "mmdx_stream_destroy");
  return 0;
}
