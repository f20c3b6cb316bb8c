// ABI bookkeeping for libsmpq: version and thread-local last error.
#include <string>

#include "common.h"

namespace smpq {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
}  // namespace smpq

// The SHA-256 of the sources, headers and flags (set by __graft_entry__.build() with
// -DSMPQ_BUILD_STAMP=<hex>); the marker prefix lets build() read it from the file unloaded.
#ifndef SMPQ_BUILD_STAMP
#define SMPQ_BUILD_STAMP "unstamped"
#endif
static const char kStamp[] = "smpq-build-stamp:" SMPQ_BUILD_STAMP;

extern "C" int smpq_abi_version(void) { return SMPQ_ABI_VERSION; }
extern "C" const char* smpq_build_stamp(void) { return kStamp + 17; }
extern "C" const char* smpq_last_error(void) { return smpq::g_last_error.c_str(); }
