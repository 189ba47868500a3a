// Library identification and the thread-local error channel of the C ABI (include/gr_amd.h).
#include <string>

#include "gr_common.h"

namespace gr {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
void clear_error() { g_last_error.clear(); }
}  // namespace gr

extern "C" const char* gr_version(void) { return "gr_amd 0.1.0 gfx950"; }
extern "C" const char* gr_last_error(void) { return gr::g_last_error.c_str(); }
