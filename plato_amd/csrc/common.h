// Internal helpers shared by the HIP translation units of libplato_agg.so
// (not part of the C ABI).
#pragma once

#include <hip/hip_runtime_api.h>

#include <mutex>
#include <string>

namespace plato_agg_internal {

// Sets the thread-local message returned by plato_agg_last_error() and
// returns `code` (a PLATO_AGG_E* status).
__attribute__((visibility("hidden"))) int set_error(int code, const std::string& msg);

// Clears the message; returns PLATO_AGG_OK.
__attribute__((visibility("hidden"))) int clear_error();

// A second stream per device (created on first use, never destroyed) with a fork / join event pair, so
// that independent launches of one C-ABI call overlap: record `fork` on the caller's stream and make `s`
// wait for it, launch on `s`, then record `join` on `s` and make the caller's stream wait for it.  The
// sequence runs under `mu` (the events are reused across calls; a wait captures an event's state when it
// is enqueued), so concurrent callers stay ordered.  Defined in flat.hip.
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  std::mutex mu;
};
__attribute__((visibility("hidden"))) SideStream* side_stream(int dev);

}  // namespace plato_agg_internal
