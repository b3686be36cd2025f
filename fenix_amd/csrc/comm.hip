// Single-process multi-GPU exchange of per-shard top-k lists over RCCL (xGMI).
//
// The serving path (one Flight server process driving every GPU of a node,
// SURVEY §8(e), configs[4]) row-shards each corpus over the devices; after the
// per-device scans, every shard's (distance, row) top-k list is all-gathered
// with ONE grouped RCCL call and merged by fx_topk_merge.  The reference is
// single-process and single-device (its select over the concatenated sources,
// src/fenix/io/table/table.py:19-21 + src/fenix/io/index/index.py:166, is what
// the gather + merge replaces).  One process per GPU uses torch.distributed
// instead (fenix_amd/distributed.py, bench.py).
//
// RCCL is opened with dlopen on first use, so the library has no link-time
// RCCL dependency; inside a torch process the already loaded librccl.so.1 is
// reused (same soname).
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <stdlib.h>
#include <string.h>

#include "fx_internal.h"

namespace fx {
namespace {

struct Rccl {
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  bool ok = false;
};

const Rccl& rccl() {
  static Rccl r = [] {
    Rccl t;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (h == nullptr) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (h == nullptr) return t;
    t.init_all = reinterpret_cast<decltype(&ncclCommInitAll)>(dlsym(h, "ncclCommInitAll"));
    t.destroy = reinterpret_cast<decltype(&ncclCommDestroy)>(dlsym(h, "ncclCommDestroy"));
    t.all_gather = reinterpret_cast<decltype(&ncclAllGather)>(dlsym(h, "ncclAllGather"));
    t.group_start = reinterpret_cast<decltype(&ncclGroupStart)>(dlsym(h, "ncclGroupStart"));
    t.group_end = reinterpret_cast<decltype(&ncclGroupEnd)>(dlsym(h, "ncclGroupEnd"));
    t.error_string =
        reinterpret_cast<decltype(&ncclGetErrorString)>(dlsym(h, "ncclGetErrorString"));
    t.ok = t.init_all && t.destroy && t.all_gather && t.group_start && t.group_end &&
           t.error_string;
    return t;
  }();
  return r;
}

constexpr int kMaxDevs = 64;

struct Comm {
  int ndev;
  int devs[kMaxDevs];
  ncclComm_t comms[kMaxDevs];
};

int rccl_error(const char* what, ncclResult_t r) {
  set_error("%s: %s", what, rccl().error_string(r));
  return FX_EHIP;
}

}  // namespace
}  // namespace fx

using namespace fx;

extern "C" {

int fx_comm_init_all(int ndev, const int* devs, void** out_comm) {
  if (out_comm == nullptr || devs == nullptr || ndev < 1 || ndev > kMaxDevs) {
    set_error("fx_comm_init_all: invalid arguments (ndev=%d)", ndev);
    return FX_EINVAL;
  }
  *out_comm = nullptr;
  for (int i = 0; i < ndev; ++i)
    for (int j = 0; j < i; ++j)
      if (devs[i] == devs[j]) {
        set_error("fx_comm_init_all: device %d listed twice (one rank per device)", devs[i]);
        return FX_EINVAL;
      }
  const Rccl& r = rccl();
  if (!r.ok) {
    set_error("RCCL (librccl.so.1) is not available: %s", dlerror());
    return FX_EUNSUPPORTED;
  }
  Comm* c = new Comm();
  c->ndev = ndev;
  memcpy(c->devs, devs, sizeof(int) * ndev);
  int cur = 0;
  (void)hipGetDevice(&cur);
  ncclResult_t e = r.init_all(c->comms, ndev, devs);
  (void)hipSetDevice(cur);
  if (e != ncclSuccess) {
    delete c;
    return rccl_error("ncclCommInitAll", e);
  }
  *out_comm = c;
  return FX_OK;
}

int fx_comm_destroy(void* comm) {
  if (comm == nullptr) return FX_OK;
  Comm* c = reinterpret_cast<Comm*>(comm);
  int rc = FX_OK;
  for (int i = 0; i < c->ndev; ++i) {
    ncclResult_t e = rccl().destroy(c->comms[i]);
    if (e != ncclSuccess && rc == FX_OK) rc = rccl_error("ncclCommDestroy", e);
  }
  delete c;
  return rc;
}

int fx_allgather_topk(void* comm, const float* const* dist, const int64_t* const* row,
                      int64_t nq, int64_t k, float* const* all_dist, int64_t* const* all_row,
                      void* const* streams) {
  if (comm == nullptr || dist == nullptr || row == nullptr || all_dist == nullptr ||
      all_row == nullptr || streams == nullptr || nq < 1 || k < 1) {
    set_error("fx_allgather_topk: invalid arguments");
    return FX_EINVAL;
  }
  Comm* c = reinterpret_cast<Comm*>(comm);
  const Rccl& r = rccl();
  const size_t count = (size_t)nq * (size_t)k;
  int cur = 0;
  (void)hipGetDevice(&cur);
  ncclResult_t e = r.group_start();
  for (int i = 0; i < c->ndev && e == ncclSuccess; ++i) {
    (void)hipSetDevice(c->devs[i]);
    hipStream_t st = reinterpret_cast<hipStream_t>(streams[i]);
    e = r.all_gather(dist[i], all_dist[i], count, ncclFloat32, c->comms[i], st);
    if (e == ncclSuccess)
      e = r.all_gather(row[i], all_row[i], count, ncclInt64, c->comms[i], st);
  }
  ncclResult_t e2 = r.group_end();
  (void)hipSetDevice(cur);
  if (e != ncclSuccess) return rccl_error("ncclAllGather", e);
  if (e2 != ncclSuccess) return rccl_error("ncclGroupEnd", e2);
  return FX_OK;
}

}  // extern "C"
