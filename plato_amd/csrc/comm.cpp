// comm.cpp — single-process RCCL communicator over the GPUs one Plato server
// drives (C ABI in include/plato_agg.h, plato_agg_comm_*).
//
// Plato's server is one process on one event loop (plato/servers/base.py:
// 323-327), so the multi-GPU engine drives every GPU of the node from that
// process: one communicator per device from ncclCommInitAll, collectives
// issued for all devices inside one ncclGroupStart/End.  The bit-exact path
// needs no reduction (parameter buckets are independent);
// the collectives assemble the new model on every GPU when it stays
// device-resident (all-gather of the result buckets over xGMI) and serve the
// client-sharded tolerance mode (reduce-scatter of partial sums).
//
// RCCL is bound at first use with dlopen("librccl.so.1"): the process
// normally has PyTorch's copy loaded already, which the loader then returns,
// so there is exactly one RCCL in the process and no link-time dependency.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <mutex>
#include <string>
#include <vector>

#include "common.h"
#include "plato_agg.h"

struct plato_agg_comm {
  std::vector<ncclComm_t> comms;
  std::vector<int> devices;
};

namespace {

struct Rccl {
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  std::string load_error;

  bool ok() const { return init_all != nullptr; }

  static const Rccl& get() {
    static Rccl* r = load();  // never destroyed: no teardown ordering at exit
    return *r;
  }

 private:
  static Rccl* load() {
    Rccl* r = new Rccl();
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      r->load_error = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
      return r;
    }
    auto sym = [&](const char* name) { return dlsym(h, name); };
    r->destroy = reinterpret_cast<decltype(r->destroy)>(sym("ncclCommDestroy"));
    r->group_start = reinterpret_cast<decltype(r->group_start)>(sym("ncclGroupStart"));
    r->group_end = reinterpret_cast<decltype(r->group_end)>(sym("ncclGroupEnd"));
    r->all_gather = reinterpret_cast<decltype(r->all_gather)>(sym("ncclAllGather"));
    r->reduce_scatter = reinterpret_cast<decltype(r->reduce_scatter)>(sym("ncclReduceScatter"));
    r->error_string = reinterpret_cast<decltype(r->error_string)>(sym("ncclGetErrorString"));
    auto init = reinterpret_cast<decltype(r->init_all)>(sym("ncclCommInitAll"));
    if (!r->destroy || !r->group_start || !r->group_end || !r->all_gather || !r->reduce_scatter ||
        !r->error_string || !init) {
      r->load_error = "librccl.so.1 lacks an expected entry point";
      return r;
    }
    r->init_all = init;
    return r;
  }
};

int rccl_fail(const Rccl& r, ncclResult_t res, const char* what) {
  return plato_agg_internal::set_error(PLATO_AGG_ERCCL, std::string(what) + ": " + r.error_string(res));
}

int need_rccl(const Rccl** out) {
  const Rccl& r = Rccl::get();
  if (!r.ok()) return plato_agg_internal::set_error(PLATO_AGG_ERCCL, r.load_error);
  *out = &r;
  return PLATO_AGG_OK;
}

// Issue one collective per device inside a group: RCCL requires the calls of
// all local ranks of a single-thread communicator to be fused.
template <class Fn>
int grouped(const Rccl& r, plato_agg_comm* c, const char* what, Fn&& per_device) {
  ncclResult_t res = r.group_start();
  if (res != ncclSuccess) return rccl_fail(r, res, what);
  ncclResult_t first = ncclSuccess;
  for (size_t g = 0; g < c->comms.size(); ++g) {
    res = per_device(int(g));
    if (res != ncclSuccess && first == ncclSuccess) first = res;
  }
  res = r.group_end();
  if (first != ncclSuccess) return rccl_fail(r, first, what);
  if (res != ncclSuccess) return rccl_fail(r, res, what);
  return plato_agg_internal::clear_error();
}

}  // namespace

extern "C" {

int plato_agg_comm_create(int ndev, const int* devices, plato_agg_comm** out) {
  if (!out || ndev < 1 || !devices) return plato_agg_internal::set_error(PLATO_AGG_EINVAL, "bad communicator arguments");
  *out = nullptr;
  for (int i = 0; i < ndev; ++i)
    for (int j = 0; j < i; ++j)
      if (devices[i] == devices[j])
        return plato_agg_internal::set_error(PLATO_AGG_EINVAL, "RCCL needs distinct devices (one rank per GPU)");
  const Rccl* r = nullptr;
  if (int rc = need_rccl(&r)) return rc;
  auto* c = new plato_agg_comm();
  c->comms.resize(size_t(ndev));
  c->devices.assign(devices, devices + ndev);
  ncclResult_t res = r->init_all(c->comms.data(), ndev, devices);
  if (res != ncclSuccess) {
    delete c;
    return rccl_fail(*r, res, "ncclCommInitAll");
  }
  *out = c;
  return plato_agg_internal::clear_error();
}

int plato_agg_comm_destroy(plato_agg_comm* comm) {
  if (!comm) return plato_agg_internal::clear_error();
  const Rccl* r = nullptr;
  if (int rc = need_rccl(&r)) return rc;
  int status = PLATO_AGG_OK;
  for (ncclComm_t c : comm->comms) {
    ncclResult_t res = r->destroy(c);
    if (res != ncclSuccess && status == PLATO_AGG_OK) status = rccl_fail(*r, res, "ncclCommDestroy");
  }
  delete comm;
  return status == PLATO_AGG_OK ? plato_agg_internal::clear_error() : status;
}

int plato_agg_comm_size(const plato_agg_comm* comm) { return comm ? int(comm->comms.size()) : 0; }

int plato_agg_comm_allgather_f32(plato_agg_comm* comm, const float* const* d_send, float* const* d_recv,
                                 size_t count, const hipStream_t* streams) {
  if (!comm || !d_send || !d_recv || !streams)
    return plato_agg_internal::set_error(PLATO_AGG_EINVAL, "bad all-gather arguments");
  const Rccl* r = nullptr;
  if (int rc = need_rccl(&r)) return rc;
  return grouped(*r, comm, "ncclAllGather", [&](int g) {
    return r->all_gather(d_send[g], d_recv[g], count, ncclFloat32, comm->comms[size_t(g)], streams[g]);
  });
}

int plato_agg_comm_reduce_scatter_f32(plato_agg_comm* comm, const float* const* d_send, float* const* d_recv,
                                      size_t count, const hipStream_t* streams) {
  if (!comm || !d_send || !d_recv || !streams)
    return plato_agg_internal::set_error(PLATO_AGG_EINVAL, "bad reduce-scatter arguments");
  const Rccl* r = nullptr;
  if (int rc = need_rccl(&r)) return rc;
  return grouped(*r, comm, "ncclReduceScatter", [&](int g) {
    return r->reduce_scatter(d_send[g], d_recv[g], count, ncclFloat32, ncclSum, comm->comms[size_t(g)],
                             streams[g]);
  });
}

}  // extern "C"
