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

extern "C" int smpq_abi_version(void) { return SMPQ_ABI_VERSION; }
extern "C" const char* smpq_last_error(void) { return smpq::g_last_error.c_str(); }
