// libkrca: version, error reporting and device queries (host-only translation unit).
#include <map>
#include <mutex>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime.h>

#include "krca_common.h"

namespace krca {
static thread_local char g_err[1024] = "";

namespace {
int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
struct NamedKnob {
  const char* name;
  int Tuning::*field;
};
const NamedKnob kKnobs[] = {
    {"KRCA_SCORE_IMPL", &Tuning::score_impl}, {"KRCA_SCORE_CHUNK", &Tuning::score_chunk},
    {"KRCA_SCORE_NT", &Tuning::score_nt},     {"KRCA_PPR_GRID", &Tuning::ppr_grid},
    {"KRCA_PPR_DICT", &Tuning::ppr_dict},
    {"KRCA_LOG_IMPL", &Tuning::log_impl},     {"KRCA_GROUP_IMPL", &Tuning::group_impl},
    {"KRCA_CORR_DEBUG", &Tuning::corr_debug},
    {"KRCA_CORR_RS_GRID", &Tuning::corr_rs_grid},
    {"KRCA_CORR_BATCH", &Tuning::corr_batch},
    {"KRCA_CORR_AMB_TILE", &Tuning::corr_amb_tile},
    {"KRCA_PPR_FUSE", &Tuning::ppr_fuse},
    {"KRCA_PPR_NT", &Tuning::ppr_nt},
    {"KRCA_PPR_XCD", &Tuning::ppr_xcd},
    {"KRCA_LOG_FUSED", &Tuning::log_fused},
    {"KRCA_CORR_RS_GROUP", &Tuning::corr_rs_group},
    {"KRCA_CORR_SIDE", &Tuning::corr_side},
    {"KRCA_CORR_RS_Q16", &Tuning::corr_rs_q16},
    {"KRCA_CORR_CAPC", &Tuning::corr_capc},
    {"KRCA_CORR_KM_EXTRA", &Tuning::corr_km_extra},
    {"KRCA_CORR_RSG_GRID", &Tuning::corr_rsg_grid},
    {"KRCA_CORR_PROJ", &Tuning::corr_proj},
    {"KRCA_CORR_PERSIST", &Tuning::corr_persist},
};
Tuning g_tune = {env_int("KRCA_SCORE_IMPL", 0), env_int("KRCA_SCORE_CHUNK", 20), env_int("KRCA_SCORE_NT", 1),
                 env_int("KRCA_PPR_GRID", 0),   env_int("KRCA_PPR_DICT", 1),     env_int("KRCA_LOG_IMPL", 0),
                 env_int("KRCA_GROUP_IMPL", 0),
                 env_int("KRCA_CORR_DEBUG", 0), env_int("KRCA_CORR_RS_GRID", 1024),
                 env_int("KRCA_CORR_BATCH", 0),   env_int("KRCA_CORR_AMB_TILE", -1),
                 env_int("KRCA_PPR_FUSE", 0), env_int("KRCA_PPR_NT", 0),
                 env_int("KRCA_PPR_XCD", 0), env_int("KRCA_LOG_FUSED", 0), env_int("KRCA_CORR_RS_GROUP", 1),
                 env_int("KRCA_CORR_SIDE", 0), env_int("KRCA_CORR_RS_Q16", 1),
                 env_int("KRCA_CORR_CAPC", 0), env_int("KRCA_CORR_KM_EXTRA", 6),
                 env_int("KRCA_CORR_RSG_GRID", 0), env_int("KRCA_CORR_PROJ", 2),
                 env_int("KRCA_CORR_PERSIST", 0)};
const NamedKnob* find_knob(const char* name) {
  if (!name) return nullptr;
  for (const NamedKnob& k : kKnobs)
    if (!strcmp(k.name, name)) return &k;
  return nullptr;
}
}  // namespace

const Tuning& tuning() { return g_tune; }
int tuning_ppr_dict() { return g_tune.ppr_dict; }  // for the plain-C++ host units (ppr_pack.cpp)

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
hipStream_t side_stream(hipStream_t st) {
  // one per thread and device, never destroyed (a thread-exit destructor could run after the HIP
  // runtime's own teardown at process exit); the fork / join events order it, so the null stream
  // is a correct (serialising) fallback.  Created on st's device, whatever device is current.
  static thread_local hipStream_t side[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  if (st && hipStreamGetDevice(st, &dev) != hipSuccess) return nullptr;
  if (dev < 0 || dev >= 64) return nullptr;
  if (!side[dev]) {
    int cur = dev;
    (void)hipGetDevice(&cur);
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return nullptr;
    if (hipStreamCreateWithFlags(&side[dev], hipStreamNonBlocking) != hipSuccess) side[dev] = nullptr;
    if (cur != dev) (void)hipSetDevice(cur);
  }
  return side[dev];
}

int64_t resident_workgroups(const void* kernel, int tpb, hipStream_t st, int fallback_per_cu) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  if (st && hipStreamGetDevice(st, &dev) != hipSuccess) (void)hipGetDevice(&dev);
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int64_t> cache;
  std::lock_guard<std::mutex> lk(mu);
  const auto key = std::make_pair(kernel, dev);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int cus = 256, per_cu = fallback_per_cu, cur = dev;
  (void)hipGetDevice(&cur);
  const bool sw = cur != dev && hipSetDevice(dev) == hipSuccess;  // the occupancy API asks the current device
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, tpb, 0) != hipSuccess || per_cu < 1)
    per_cu = fallback_per_cu;
  if (sw) (void)hipSetDevice(cur);
  return cache[key] = (int64_t)cus * per_cu;
}
}  // namespace krca

extern "C" {

int krca_version(void) { return 100; }  // 0.1.0

const char* krca_last_error(void) { return krca::g_err; }

int krca_tune_set(const char* name, int32_t value) {
  const krca::NamedKnob* k = krca::find_knob(name);
  KRCA_CHECK_ARG(k, "krca_tune_set: unknown knob '%s'", name ? name : "(null)");
  krca::g_tune.*(k->field) = value;
  return KRCA_OK;
}

int krca_tune_get(const char* name, int32_t* value_host) {
  const krca::NamedKnob* k = krca::find_knob(name);
  KRCA_CHECK_ARG(k && value_host, "krca_tune_get: unknown knob '%s' or null out pointer", name ? name : "(null)");
  *value_host = krca::g_tune.*(k->field);
  return KRCA_OK;
}

int krca_device_count(int* n_host) {
  KRCA_CHECK_ARG(n_host != nullptr, "krca_device_count: null out pointer");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *n_host = 0;
    krca::set_error("hipGetDeviceCount: %s", hipGetErrorString(e));
    return KRCA_EDEVICE;
  }
  *n_host = n;
  return KRCA_OK;
}

}  // extern "C"
