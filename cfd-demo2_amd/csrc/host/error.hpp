// Thread-local error string behind cfd_last_error().
#pragma once
#include <string>

#include "../../../include/cfd2_amd.h"

namespace cfd2 {
cfd_status set_error(cfd_status st, const std::string& msg);
}
