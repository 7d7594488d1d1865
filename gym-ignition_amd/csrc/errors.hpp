// errors.hpp -- the thread-local last error behind mw_last_error() (sim.cpp).
#pragma once

#include <string>

namespace mw {
void set_last_error(const std::string& msg);
}  // namespace mw
