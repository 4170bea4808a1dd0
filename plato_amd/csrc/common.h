// Internal helpers shared by the HIP translation units of libplato_agg.so
// (not part of the C ABI).
#pragma once

#include <string>

namespace plato_agg_internal {

// Sets the thread-local message returned by plato_agg_last_error() and
// returns `code` (a PLATO_AGG_E* status).
__attribute__((visibility("hidden"))) int set_error(int code, const std::string& msg);

// Clears the message; returns PLATO_AGG_OK.
__attribute__((visibility("hidden"))) int clear_error();

}  // namespace plato_agg_internal
