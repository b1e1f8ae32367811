// dcn_comm.cpp — data-parallel gradient exchange for batch-sharded DeformConv2d
// (SURVEY §8(e)): ONE in-place sum all-reduce of the packed parameter gradients
// (∂W, ∂b, ∂W_off, ∂b_off: 631,570 fp32 = 2.53 MB at config 3) per step, on the
// handle's stream, over RCCL (xGMI between the GPUs of one node).
//
// The reference trains on one device (train.py:414 optimizer.backward), so there is no
// reference call to mirror; this is the exchange step a multi-GPU caller that has no
// torch.distributed (the Jittor / NumPy drop-in) needs. RCCL is opened with dlopen on
// first use: libdcn carries no link-time RCCL dependency, and a process that already
// holds an RCCL (e.g. torch's) reuses that copy instead of loading a second one.
#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "dcn_internal.h"

extern "C" __attribute__((visibility("hidden"))) int dcn_internal_fail(int code, const char* msg);
extern "C" __attribute__((visibility("hidden"))) int dcn_internal_bind(dcn_handle* h,
                                                                      void** stream);
extern "C" __attribute__((visibility("hidden"))) int dcn_internal_allreduce(
    dcn_comm* c, void* buf, size_t count, int dtype, void* st);

namespace {

// The RCCL/NCCL C API subset used here (rccl.h): opaque comm, 128-byte unique id.
typedef struct ncclComm* ncclComm_t;
struct ncclUniqueId {
  char internal[DCN_COMM_ID_BYTES];
};
typedef int (*GetUniqueId_t)(ncclUniqueId*);
typedef int (*CommInitRank_t)(ncclComm_t*, int, ncclUniqueId, int);
typedef int (*CommDestroy_t)(ncclComm_t);
typedef int (*AllReduce_t)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t);
typedef const char* (*GetErrorString_t)(int);
typedef int (*Group_t)(void);
constexpr int kNcclFloat32 = 7;   // ncclFloat32
constexpr int kNcclBfloat16 = 9;  // ncclBfloat16
constexpr int kNcclSum = 0;       // ncclSum

struct Rccl {
  void* lib = nullptr;
  GetUniqueId_t get_id = nullptr;
  CommInitRank_t init = nullptr;
  CommDestroy_t destroy = nullptr;
  AllReduce_t allreduce = nullptr;
  GetErrorString_t errstr = nullptr;
  Group_t group_start = nullptr, group_end = nullptr;
};

Rccl* rccl(std::string* err) {
  static Rccl r;
  static bool tried = false;
  if (!tried) {
    tried = true;
    // An RCCL already in the process (torch's own copy, whose NEEDED name is librccl.so)
    // is reused as is. Otherwise one is loaded RTLD_LOCAL: with RTLD_GLOBAL, a second copy
    // that torch loads later (libtorch_hip NEEDs "librccl.so", not the "librccl.so.1" this
    // loads) bound its symbols into ours, and the process aborted at exit with a corrupted
    // heap (r02, test_gpu_configs.py run alone, torch imported after the first comm test).
    for (const char* name : {"librccl.so", "librccl.so.1"}) {
      r.lib = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
      if (r.lib) break;
    }
    if (!r.lib)
      for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
        r.lib = dlopen(name, RTLD_NOW | RTLD_LOCAL);
        if (r.lib) break;
      }
    if (r.lib) {
      r.get_id = (GetUniqueId_t)dlsym(r.lib, "ncclGetUniqueId");
      r.init = (CommInitRank_t)dlsym(r.lib, "ncclCommInitRank");
      r.destroy = (CommDestroy_t)dlsym(r.lib, "ncclCommDestroy");
      r.allreduce = (AllReduce_t)dlsym(r.lib, "ncclAllReduce");
      r.errstr = (GetErrorString_t)dlsym(r.lib, "ncclGetErrorString");
      r.group_start = (Group_t)dlsym(r.lib, "ncclGroupStart");
      r.group_end = (Group_t)dlsym(r.lib, "ncclGroupEnd");
    }
  }
  if (!r.lib || !r.get_id || !r.init || !r.destroy || !r.allreduce || !r.group_start ||
      !r.group_end) {
    *err = "RCCL (librccl.so.1) not loadable";
    return nullptr;
  }
  return &r;
}

int rccl_fail(Rccl* r, const char* what, int rc) {
  std::string m = std::string(what) + " failed: " + (r->errstr ? r->errstr(rc) : "") + " (" +
                  std::to_string(rc) + ")";
  return dcn_internal_fail(DCN_ERR_COMM, m.c_str());
}

}  // namespace

struct dcn_comm {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0;
  // handles this communicator is attached to (dcn_set_comm): dcn_comm_destroy detaches
  // them first, so no handle keeps a dangling pointer or races an in-flight exchange
  std::vector<dcn_handle*> users;
};

extern "C" __attribute__((visibility("hidden"))) void dcn_internal_handle_drop_comm(dcn_handle* h);

extern "C" __attribute__((visibility("hidden"))) void dcn_internal_comm_attach(dcn_comm* c,
                                                                             dcn_handle* h) {
  if (c && std::find(c->users.begin(), c->users.end(), h) == c->users.end())
    c->users.push_back(h);
}
extern "C" __attribute__((visibility("hidden"))) void dcn_internal_comm_detach(dcn_comm* c,
                                                                             dcn_handle* h) {
  if (c) c->users.erase(std::remove(c->users.begin(), c->users.end(), h), c->users.end());
}

extern "C" {

int dcn_comm_get_unique_id(void* id) {
  if (!id) return dcn_internal_fail(DCN_ERR_INVALID, "null id buffer");
  std::string err;
  Rccl* r = rccl(&err);
  if (!r) return dcn_internal_fail(DCN_ERR_COMM, err.c_str());
  ncclUniqueId u;
  const int rc = r->get_id(&u);
  if (rc != 0) return rccl_fail(r, "ncclGetUniqueId", rc);
  std::memcpy(id, u.internal, DCN_COMM_ID_BYTES);
  return DCN_OK;
}

int dcn_comm_init(dcn_handle* h, int nranks, int rank, const void* id, dcn_comm** out) {
  if (!out || !id) return dcn_internal_fail(DCN_ERR_INVALID, "null argument");
  *out = nullptr;
  if (nranks < 1 || rank < 0 || rank >= nranks)
    return dcn_internal_fail(DCN_ERR_INVALID, "rank out of range");
  void* st = nullptr;
  int rc = dcn_internal_bind(h, &st);  // selects the handle's device
  if (rc != DCN_OK) return rc;
  std::string err;
  Rccl* r = rccl(&err);
  if (!r) return dcn_internal_fail(DCN_ERR_COMM, err.c_str());
  ncclUniqueId u;
  std::memcpy(u.internal, id, DCN_COMM_ID_BYTES);
  dcn_comm* c = new dcn_comm();
  rc = r->init(&c->comm, nranks, u, rank);
  if (rc != 0) {
    delete c;
    return rccl_fail(r, "ncclCommInitRank", rc);
  }
  c->nranks = nranks;
  c->rank = rank;
  *out = c;
  return DCN_OK;
}

int dcn_comm_destroy(dcn_comm* c) {
  if (!c) return DCN_OK;
  // waits for each attached handle's exchange stream, then clears its pointer
  while (!c->users.empty()) dcn_internal_handle_drop_comm(c->users.back());
  std::string err;
  Rccl* r = rccl(&err);
  if (r && c->comm) r->destroy(c->comm);
  delete c;
  return DCN_OK;
}

int dcn_allreduce_grads(dcn_handle* h, dcn_comm* c, void* grads, size_t count, int dtype) {
  if (!c || (!grads && count)) return dcn_internal_fail(DCN_ERR_INVALID, "null argument");
  if (dtype != DCN_F32 && dtype != DCN_BF16)
    return dcn_internal_fail(DCN_ERR_INVALID, "dcn_allreduce_grads: dtype must be DCN_F32 or DCN_BF16");
  void* st = nullptr;
  int rc = dcn_internal_bind(h, &st);
  if (rc != DCN_OK) return rc;
  if (count == 0) return DCN_OK;
  // the buffer must hold count elements of dtype inside ONE device allocation (a count in
  // fp32 elements over a bf16 buffer would run RCCL 2x past its end)
  const size_t bytes = count * (dtype == DCN_BF16 ? 2 : 4);
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, grads) != hipSuccess || !base)
    return dcn_internal_fail(DCN_ERR_INVALID, "dcn_allreduce_grads: grads is not device memory");
  const char* b = static_cast<const char*>(base);
  const char* p = static_cast<const char*>(grads);
  if (p + bytes > b + size)
    return dcn_internal_fail(DCN_ERR_INVALID,
                             "dcn_allreduce_grads: count x sizeof(dtype) runs past the end of "
                             "the allocation holding grads");
  return dcn_internal_allreduce(c, grads, count, dtype, st);
}

}  // extern "C"

// In-place sums for dcn_backward when a communicator is attached (dcn_set_comm): several
// buffers in one RCCL group, on stream st. Internal (not in dcn.h).
extern "C" __attribute__((visibility("hidden"))) int dcn_internal_allreduce_n(
    dcn_comm* c, int n, void* const* bufs, const size_t* counts, int dtype, void* st) {
  std::string err;
  Rccl* r = rccl(&err);
  if (!r) return dcn_internal_fail(DCN_ERR_COMM, err.c_str());
  const int ty = dtype == DCN_BF16 ? kNcclBfloat16 : kNcclFloat32;
  int rc = r->group_start();
  if (rc != 0) return rccl_fail(r, "ncclGroupStart", rc);
  for (int i = 0; i < n; ++i) {
    if (!counts[i]) continue;
    rc = r->allreduce(bufs[i], bufs[i], counts[i], ty, kNcclSum, c->comm,
                      static_cast<hipStream_t>(st));
    if (rc != 0) {
      (void)r->group_end();
      return rccl_fail(r, "ncclAllReduce", rc);
    }
  }
  rc = r->group_end();
  if (rc != 0) return rccl_fail(r, "ncclGroupEnd", rc);
  return DCN_OK;
}

extern "C" __attribute__((visibility("hidden"))) int dcn_internal_allreduce(
    dcn_comm* c, void* buf, size_t count, int dtype, void* st) {
  return dcn_internal_allreduce_n(c, 1, &buf, &count, dtype, st);
}
