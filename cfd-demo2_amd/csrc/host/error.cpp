// Thread-local error string behind cfd_last_error().
#include "error.hpp"

namespace cfd2 {
static thread_local std::string g_last_error;
cfd_status set_error(cfd_status st, const std::string& msg) {
  g_last_error = msg;
  return st;
}
}  // namespace cfd2

extern "C" const char* cfd_last_error(void) { return cfd2::g_last_error.c_str(); }
