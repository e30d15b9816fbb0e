// Host-side plumbing of the C ABI: error reporting and version.
#include "aon_common.hpp"

namespace aon {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace aon

extern "C" int aon_abi_version(void) { return AON_ABI_VERSION; }

extern "C" const char* aon_last_error(void) { return aon::g_last_error.c_str(); }
