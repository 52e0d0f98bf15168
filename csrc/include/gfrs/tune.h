// GFRS_TUNE: the one switchboard for launch thresholds and measurement aids.
//
// Every tuned constant of the native code has a measured default (cited where it is used); a
// measurement run overrides them through one variable, "key=value" pairs separated by commas:
//
//   GFRS_TUNE=fp4=tm,ksplit_lanes=0 python bench.py --preset k128n160
//
// Keys (docs/API.md lists them with their defaults): fp4 (v1 | ar | tm: force a GF(2^8) FP4 kernel
// form where it is built), tm8, rows_lat_groups, ksplit_lanes, short_lanes, vec_cfg (V:PF:NT), gf16_vec_g,
// gf16_short_groups, fp16_mg, fp4_free_cus, max_rect_pitch, zc_stream (own), setup (serial), crc
// (scalar). Unknown keys are ignored. Besides GFRS_TUNE the native code reads only GFRS_HOST_ALLOC
// and GFRS_VERIFY_THREADS (operational choices, not tuning).
#pragma once

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>

namespace gfrs {

// value of `key` in GFRS_TUNE, or "" when absent (parsed on every call: tests and A/B runs switch
// it inside one process; call sites that take it once per process cache the result themselves)
inline std::string tune_str(const char* key) {
  const char* env = std::getenv("GFRS_TUNE");
  if (!env || !*env) return {};
  const size_t klen = std::strlen(key);
  for (const char* p = env; *p;) {
    const char* end = std::strchr(p, ',');
    if (!end) end = p + std::strlen(p);
    const char* eq = static_cast<const char*>(std::memchr(p, '=', size_t(end - p)));
    if (eq && size_t(eq - p) == klen && std::strncmp(p, key, klen) == 0) return std::string(eq + 1, end);
    p = *end ? end + 1 : end;
  }
  return {};
}

inline int64_t tune_int(const char* key, int64_t dflt) {
  const std::string v = tune_str(key);
  if (v.empty()) return dflt;
  char* end = nullptr;
  const long long x = std::strtoll(v.c_str(), &end, 10);
  return end && *end == '\0' ? int64_t(x) : dflt;
}

}  // namespace gfrs
