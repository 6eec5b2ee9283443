// transport.cpp -- RCCL communicators the engine drives itself (ABI 7; include/dopt.h "Engine-driven
// RCCL transport").  The lagged schedule's per-round exchange (distributed.py _run_lagged; the reference's
// neighbour reads of W @ X, trainer.py:173) went through torch's process group: ~22 us of host time per
// call for alltoall_base and 36-40 us with its work.wait() (profiles/r5_rccl_probe.txt), where RCCL's own
// group of point-to-point calls costs 4.5-6 us on the same box.  A dopt_comm is an RCCL communicator over
// the job's ranks; dopt_lagged_exchange (runtime.cpp) issues a round's sends and receives through it
// directly on the context's side stream.
//
// Every blocking step is bounded (ABI 8): the communicator is created NON-blocking
// (ncclCommInitRankConfig, config.blocking = 0) and its setup polled with ncclCommGetAsyncError until done
// or until the caller's timeout, then aborted -- a rank that never joins costs the others DOPT_ERR_COMM
// after timeout_s instead of a hang in ncclCommInitRank.  On such a communicator ncclGroupEnd may return
// ncclInProgress while RCCL connects a new peer in the background (the first exchange with each peer):
// comm_exchange then polls, under the same bound, until the sends / receives are enqueued on the stream,
// so on return they are ordered before whatever the caller records on it next.
//
// RCCL is resolved at run time: the copy already in the process (torch's bundled librccl.so, the same
// library its process group uses) when there is one, else librccl.so.1 (DOPT_RCCL_LIB overrides), so
// the library has no link-time dependency on either.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <mutex>
#include <thread>
#include <new>
#include <string>
#include <type_traits>

#include "dopt.h"
#include "engine.h"

struct dopt_comm {
  ncclComm_t comm = nullptr;
  int32_t world = 0, rank = 0, device = 0;
  double timeout_s = 0.0;  // bound on every host wait for RCCL (setup, a peer's first connection, destroy)
};

namespace {

struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRankConfig) init_rank_config = nullptr;
  decltype(&ncclCommFinalize) finalize = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommAbort) abort = nullptr;
  decltype(&ncclCommGetAsyncError) async_error = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  std::string path, err;
};

const Rccl* rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    const char* over = getenv("DOPT_RCCL_LIB");
    if (over && *over) {
      h = dlopen(over, RTLD_NOW | RTLD_LOCAL);
    } else {
      h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);  // torch's copy, when torch is loaded
      if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
      if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    }
    if (!h) {
      r.err = std::string("RCCL not found: ") + dlerror();
      return;
    }
    Dl_info info;
    bool ok = true;
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      if (!fn) ok = false;
    };
    sym(r.get_unique_id, "ncclGetUniqueId");
    sym(r.init_rank_config, "ncclCommInitRankConfig");
    sym(r.finalize, "ncclCommFinalize");
    sym(r.destroy, "ncclCommDestroy");
    sym(r.abort, "ncclCommAbort");
    sym(r.async_error, "ncclCommGetAsyncError");
    sym(r.error_string, "ncclGetErrorString");
    sym(r.group_start, "ncclGroupStart");
    sym(r.group_end, "ncclGroupEnd");
    sym(r.send, "ncclSend");
    sym(r.recv, "ncclRecv");
    if (!ok) {
      r.err = "RCCL library lacks a required symbol";
      r.get_unique_id = nullptr;
      return;
    }
    r.path = dladdr((void*)r.send, &info) && info.dli_fname ? info.dli_fname : "?";
  });
  return &r;
}

int comm_fail(const char* what, ncclResult_t rc) {
  const Rccl* r = rccl();
  return dopt::fail_code(DOPT_ERR_COMM, "%s: %s", what, r->error_string ? r->error_string(rc) : "RCCL error");
}

#define RCCLOK(call, what)                             \
  do {                                                 \
    ncclResult_t rc_ = (call);                         \
    if (rc_ != ncclSuccess) return comm_fail(what, rc_); \
  } while (0)

const Rccl* rccl_or_fail(int* rc) {
  const Rccl* r = rccl();
  *rc = r->get_unique_id ? DOPT_OK : dopt::fail_code(DOPT_ERR_COMM, "%s", r->err.c_str());
  return r;
}

// Poll a non-blocking communicator until its pending operation (setup, a group's launch, finalize) has
// completed: DOPT_OK; RCCL's error; or, past timeout_s (<= 0: unbounded), DOPT_ERR_COMM with *timed_out set.
// The wait backs off from 20 us to 1 ms per poll (a group launch completes in microseconds, a setup in
// hundreds of milliseconds).
int poll_ready(const Rccl* r, ncclComm_t comm, double timeout_s, const char* what, bool* timed_out) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  auto nap = std::chrono::microseconds(20);
  *timed_out = false;
  for (;;) {
    ncclResult_t async = ncclSuccess;
    const ncclResult_t q = r->async_error(comm, &async);
    if (q != ncclSuccess) return comm_fail("ncclCommGetAsyncError", q);
    if (async == ncclSuccess) return DOPT_OK;
    if (async != ncclInProgress) return comm_fail(what, async);
    const double el = std::chrono::duration<double>(clk::now() - t0).count();
    if (timeout_s > 0 && el > timeout_s) {
      *timed_out = true;
      return dopt::fail_code(DOPT_ERR_COMM, "%s did not complete in %.0f s (a peer never joined?)", what, timeout_s);
    }
    std::this_thread::sleep_for(nap);
    nap = std::min(nap * 2, std::chrono::microseconds(1000));
  }
}

}  // namespace

namespace dopt {

int comm_exchange(dopt_comm* c, const XpOp* ops, size_t n_ops, const void* send, void* recv, hipStream_t s) {
  int rc;
  const Rccl* r = rccl_or_fail(&rc);
  if (rc) return rc;
  RCCLOK(r->group_start(), "ncclGroupStart");
  ncclResult_t st = ncclSuccess;
  for (size_t k = 0; k < n_ops && st == ncclSuccess; ++k) {
    const XpOp& o = ops[k];
    st = o.recv ? r->recv((char*)recv + o.off, (size_t)o.bytes, ncclInt8, o.peer, c->comm, s)
                : r->send((const char*)send + o.off, (size_t)o.bytes, ncclInt8, o.peer, c->comm, s);
  }
  const ncclResult_t end = r->group_end();  // (closes the group whatever the sends returned)
  if (st != ncclSuccess && st != ncclInProgress) return comm_fail("ncclSend / ncclRecv", st);
  if (end == ncclInProgress) {  // a new peer being connected in the background: wait until enqueued
    bool timed_out = false;
    return poll_ready(r, c->comm, c->timeout_s, "the exchange's first connection to a peer", &timed_out);
  }
  if (end != ncclSuccess) return comm_fail("ncclGroupEnd", end);
  return DOPT_OK;
}

int32_t comm_world(const dopt_comm* c) { return c->world; }
int32_t comm_rank(const dopt_comm* c) { return c->rank; }
int32_t comm_device(const dopt_comm* c) { return c->device; }

}  // namespace dopt

extern "C" {

int dopt_comm_unique_id(uint8_t* id_out, int64_t n) {
  if (!id_out || n < DOPT_COMM_ID_BYTES) return dopt::fail_code(DOPT_ERR_INVALID, "id buffer of %d bytes needed", DOPT_COMM_ID_BYTES);
  static_assert(sizeof(ncclUniqueId) == DOPT_COMM_ID_BYTES, "RCCL unique id size");
  int rc;
  const Rccl* r = rccl_or_fail(&rc);
  if (rc) return rc;
  ncclUniqueId id;
  RCCLOK(r->get_unique_id(&id), "ncclGetUniqueId");
  memcpy(id_out, &id, sizeof(id));
  return DOPT_OK;
}

int dopt_comm_create(dopt_comm** out, int32_t world, int32_t rank, int32_t device, const uint8_t* id, int64_t n,
                     double timeout_s) {
  if (!out || !id || n < DOPT_COMM_ID_BYTES) return dopt::fail_code(DOPT_ERR_INVALID, "NULL argument or short id");
  if (world < 1 || rank < 0 || rank >= world) return dopt::fail_code(DOPT_ERR_INVALID, "bad world %d / rank %d", world, rank);
  if (!(timeout_s >= 0)) return dopt::fail_code(DOPT_ERR_INVALID, "timeout_s must be >= 0 (0: unbounded)");
  *out = nullptr;
  int rc;
  const Rccl* r = rccl_or_fail(&rc);
  if (rc) return rc;
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess)
    return dopt::fail_code(DOPT_ERR_HIP, "hipSetDevice(%d) failed", device);
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t comm = nullptr;
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;  // returns at once; the setup (collective: every rank of the job) is polled below
  const ncclResult_t st = r->init_rank_config(&comm, world, uid, rank, &cfg);
  if (st != ncclSuccess && st != ncclInProgress) {
    if (comm) r->abort(comm);
    (void)hipSetDevice(prev);
    return comm_fail("ncclCommInitRankConfig", st);
  }
  bool timed_out = false;
  rc = poll_ready(r, comm, timeout_s, "RCCL communicator setup (ncclCommInitRankConfig)", &timed_out);
  if (rc != DOPT_OK) {
    r->abort(comm);  // (also ends an unfinished setup: its bootstrap thread and sockets)
    (void)hipSetDevice(prev);
    return rc;
  }
  (void)hipSetDevice(prev);
  dopt_comm* c = new (std::nothrow) dopt_comm;
  if (!c) {
    r->abort(comm);
    return dopt::fail_code(DOPT_ERR_NOMEM, "out of host memory");
  }
  c->comm = comm;
  c->world = world;
  c->rank = rank;
  c->device = device;
  c->timeout_s = timeout_s;
  *out = c;
  return DOPT_OK;
}

int dopt_comm_check(dopt_comm* c) {
  if (!c) return dopt::fail_code(DOPT_ERR_INVALID, "comm is NULL");
  int rc;
  const Rccl* r = rccl_or_fail(&rc);
  if (rc) return rc;
  ncclResult_t async = ncclSuccess;
  RCCLOK(r->async_error(c->comm, &async), "ncclCommGetAsyncError");
  if (async != ncclSuccess && async != ncclInProgress) return comm_fail("RCCL asynchronous error", async);
  return DOPT_OK;
}

int dopt_comm_destroy(dopt_comm* c, int32_t abort) {
  if (!c) return DOPT_OK;
  int rc;
  const Rccl* r = rccl_or_fail(&rc);
  if (rc) return rc;
  ncclComm_t comm = c->comm;
  const double timeout_s = c->timeout_s;
  delete c;
  if (abort) {
    const ncclResult_t st = r->abort(comm);
    return st == ncclSuccess ? DOPT_OK : comm_fail("ncclCommAbort", st);
  }
  // a non-blocking communicator finalizes in the background (its pending operations flushed): polled under
  // the same bound, then destroyed; a finalize that cannot complete (a peer gone) ends in an abort
  ncclResult_t st = r->finalize(comm);
  if (st == ncclSuccess || st == ncclInProgress) {
    bool timed_out = false;
    rc = poll_ready(r, comm, timeout_s, "ncclCommFinalize", &timed_out);
    if (rc != DOPT_OK) {
      r->abort(comm);
      return rc;
    }
    st = r->destroy(comm);
    return st == ncclSuccess ? DOPT_OK : comm_fail("ncclCommDestroy", st);
  }
  r->abort(comm);
  return comm_fail("ncclCommFinalize", st);
}

const char* dopt_comm_library(void) {
  const Rccl* r = rccl();
  return r->get_unique_id ? r->path.c_str() : "";
}

}  // extern "C"
