// ABI bookkeeping: version and thread-local last-error string.
#include "common.hpp"

namespace nt {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
void clear_error() { g_last_error.clear(); }
// the layer kernel variant the last layer call on this thread launched (static strings only)
static thread_local const char* g_last_kernel = "";
void set_last_kernel(const char* name) { g_last_kernel = name; }
}  // namespace nt

extern "C" int nt_abi_version(void) { return NT_ABI_VERSION; }

extern "C" const char* nt_last_error(void) { return nt::g_last_error.c_str(); }

extern "C" const char* nt_last_kernel(void) { return nt::g_last_kernel; }
