// C-ABI status plumbing for libhvk: error codes + last-error text (thread-local).
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "hvk_common.h"
#include "../../include/hvk.h"

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

int hvk_abi_version(void) { return HVK_ABI_VERSION; }

}  // extern "C"

namespace {
struct OptDef {
  const char* name;
  long long value, lo, hi;
};
OptDef g_opts[HVK_OPT_COUNT] = {
    {"wmsa_fwd_form", 0, 0, 1},
    {"wmsa_bwd_nt", 0, 0, 2},
    {"wmsa_bwd_slice_bytes", 1ll << 31, 1, 1ll << 31},
    {"tile_wide", -1, -1, 1},
    {"dw_tile", 5, 4, 8},
    {"wmsa_fwd_hg", 0, 0, 6},
    {"dw_chunks", 256, 16, 1024},
};
int find_opt(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < HVK_OPT_COUNT; ++i)
    if (!strcmp(g_opts[i].name, name)) return i;
  return -1;
}
}  // namespace

long long hvk_opt(int id) { return g_opts[id].value; }

extern "C" {

int hvk_set_option(const char* name, long long value, long long* previous) {
  const int i = find_opt(name);
  if (i < 0) return hvk_set_error(HVK_EINVAL, "hvk_set_option: unknown option '%s'", name ? name : "(null)");
  if (value < g_opts[i].lo || value > g_opts[i].hi)
    return hvk_set_error(HVK_EINVAL, "hvk_set_option: %s = %lld not in [%lld, %lld]", name, value,
                         g_opts[i].lo, g_opts[i].hi);
  if (previous) *previous = g_opts[i].value;
  g_opts[i].value = value;
  return HVK_OK;
}

int hvk_get_option(const char* name, long long* value) {
  const int i = find_opt(name);
  if (i < 0) return hvk_set_error(HVK_EINVAL, "hvk_get_option: unknown option '%s'", name ? name : "(null)");
  if (!value) return hvk_set_error(HVK_EINVAL, "hvk_get_option: null pointer");
  *value = g_opts[i].value;
  return HVK_OK;
}

// ---- kernel timer ------------------------------------------------------------------
namespace {
struct TimerShape {
  char name[48];  // "family<epi,tile>"; empty: no shape recorded
  double mnk[3], bytes;
};
struct TimerRec {
  int kind;
  double work;
  hipEvent_t start, stop;
  TimerShape shape;
};
TimerShape g_pending_shape{};
std::vector<TimerRec> g_timer;  // event pool (created once, reused)
size_t g_timer_used = 0;
bool g_timer_on = false;
int g_timer_kinds = 0xF;  // bit k: time launches of kind k
}  // namespace

void hvk_timer_next(int kind, double work, hipEvent_t* start, hipEvent_t* stop) {
  if (!g_timer_on || !((g_timer_kinds >> kind) & 1) || g_timer_used >= g_timer.size()) {
    *start = *stop = nullptr;
    return;
  }
  TimerRec& r = g_timer[g_timer_used++];
  r.kind = kind;
  r.work = work;
  r.shape = g_pending_shape;
  g_pending_shape.name[0] = 0;
  *start = r.start;
  *stop = r.stop;
}

void hvk_timer_shape(const char* family, int epi, int tile, double m, double n, double k, double bytes) {
  if (!g_timer_on) return;
  snprintf(g_pending_shape.name, sizeof(g_pending_shape.name), "%s<%d,%d>", family, epi, tile);
  g_pending_shape.mnk[0] = m;
  g_pending_shape.mnk[1] = n;
  g_pending_shape.mnk[2] = k;
  g_pending_shape.bytes = bytes;
}

int hvk_kernel_timer_enable(int max_launches) {
  g_timer_used = 0;
  g_timer_on = max_launches > 0;
  while (g_timer.size() < (size_t)(max_launches > 0 ? max_launches : 0)) {
    TimerRec r{-1, 0.0, nullptr, nullptr, {}};
    if (hipEventCreate(&r.start) != hipSuccess || hipEventCreate(&r.stop) != hipSuccess)
      return hvk_set_error(HVK_EHIP, "hvk_kernel_timer_enable: hipEventCreate failed");
    g_timer.push_back(r);
  }
  return HVK_OK;
}

int hvk_kernel_timer_kinds(int mask) {
  g_timer_kinds = mask;
  return HVK_OK;
}

int hvk_kernel_timer_read_work(int kind, double* total_ms, int* launches, double* work) {
  if (!total_ms || !launches) return hvk_set_error(HVK_EINVAL, "hvk_kernel_timer_read: null pointer");
  double t = 0.0, w = 0.0;
  int n = 0;
  for (size_t i = 0; i < g_timer_used; ++i) {
    const TimerRec& r = g_timer[i];
    if (r.kind != kind) continue;
    float ms = 0.f;
    if (hipEventSynchronize(r.stop) != hipSuccess || hipEventElapsedTime(&ms, r.start, r.stop) != hipSuccess)
      return hvk_set_error(HVK_EHIP, "hvk_kernel_timer_read: event query failed");
    t += ms;
    w += r.work;
    ++n;
  }
  *total_ms = t;
  *launches = n;
  if (work) *work = w;
  return HVK_OK;
}

int hvk_kernel_timer_launch(int index, int* kind, double* ms, double* work) {
  if (!kind || !ms) return hvk_set_error(HVK_EINVAL, "hvk_kernel_timer_launch: null pointer");
  if (index < 0 || (size_t)index >= g_timer_used)
    return hvk_set_error(HVK_EINVAL, "hvk_kernel_timer_launch: index %d of %zu", index, g_timer_used);
  const TimerRec& r = g_timer[index];
  float t = 0.f;
  if (hipEventSynchronize(r.stop) != hipSuccess || hipEventElapsedTime(&t, r.start, r.stop) != hipSuccess)
    return hvk_set_error(HVK_EHIP, "hvk_kernel_timer_launch: event query failed");
  *kind = r.kind;
  *ms = t;
  if (work) *work = r.work;
  return HVK_OK;
}

int hvk_kernel_timer_launch_shape(int index, char* name, int name_cap, double* mnk, double* bytes) {
  if (!name || name_cap < 1 || !mnk || !bytes)
    return hvk_set_error(HVK_EINVAL, "hvk_kernel_timer_launch_shape: null pointer");
  if (index < 0 || (size_t)index >= g_timer_used)
    return hvk_set_error(HVK_EINVAL, "hvk_kernel_timer_launch_shape: index %d of %zu", index, g_timer_used);
  const TimerShape& s = g_timer[index].shape;
  snprintf(name, (size_t)name_cap, "%s", s.name);
  for (int i = 0; i < 3; ++i) mnk[i] = s.mnk[i];
  *bytes = s.bytes;
  return HVK_OK;
}

int hvk_kernel_timer_read(int kind, double* total_ms, int* launches) {
  return hvk_kernel_timer_read_work(kind, total_ms, launches, nullptr);
}

}  // extern "C"
