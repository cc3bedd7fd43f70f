// C-ABI of the view-sharded path's collectives (include/mapa.h mapa_comm_*): the per-global-layer K/V all-gather and
// the scale-token broadcast over RCCL (xGMI between the GPUs of a node), so a host of libmapa.so that is not Python
// can drive the sharded forward.  Replaces the reference's process-group setup for multi-GPU runs
// (mapanything/utils/train_tools.py:389-402: torch.distributed.init_process_group("nccl") + the collectives torch
// issues on it); the Python engine's own binding of the same protocol is mapanything/rccl.py.
//
// RCCL is loaded at run time (dlopen, RTLD_LOCAL: libmapa.so keeps no link-time dependency on it, and a process that
// already holds another RCCL — torch's bundled copy — keeps both apart).  The communicator is created NON-BLOCKING
// (ncclCommInitRankConfig, blocking = 0) and its set-up polled with ncclCommGetAsyncError against the caller's
// timeout, so a rank whose peers never arrive returns an error instead of hanging in the init; a timed-out or failed
// init aborts the half-built communicator.  Every collective is enqueued on the caller's stream (capturable into a
// HIP graph with the kernels around it).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mapa_common.h"

namespace {

struct RcclApi {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRankConfig)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*) = nullptr;
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*CommFinalize)(ncclComm_t) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

// The RCCL the header describes (the ROCm image's), or MAPA_RCCL_LIB.  Loaded once; nullptr + message on failure.
const RcclApi* rccl() {
  static RcclApi api;
  static int state = 0;  // 0 not tried, 1 ok, -1 failed
  if (state == 0) {
    const char* path = getenv("MAPA_RCCL_LIB");
    if (!path) path = "/opt/rocm/lib/librccl.so.1";
    api.h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    bool ok = api.h != nullptr;
#define MAPA_SYM(F)                                                          \
  if (ok) {                                                                  \
    api.F = reinterpret_cast<decltype(api.F)>(dlsym(api.h, "nccl" #F));      \
    ok = api.F != nullptr;                                                   \
  }
    MAPA_SYM(GetUniqueId)
    MAPA_SYM(CommInitRankConfig)
    MAPA_SYM(CommGetAsyncError)
    MAPA_SYM(AllGather)
    MAPA_SYM(Broadcast)
    MAPA_SYM(CommAbort)
    MAPA_SYM(CommFinalize)
    MAPA_SYM(CommDestroy)
    MAPA_SYM(GetErrorString)
#undef MAPA_SYM
    state = ok ? 1 : -1;
    if (!ok) mapa_set_error("mapa_comm: cannot load RCCL from %s (%s)", path, dlerror());
  }
  return state == 1 ? &api : nullptr;
}

double now_s() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

}  // namespace

struct mapa_comm {
  ncclComm_t c = nullptr;
  int world = 0, rank = 0, device = 0;
  double timeout_s = 600.0;
};

// Poll the communicator's pending operation (init, a non-blocking launch) until done; abort on error / timeout.
static int comm_wait(mapa_comm* m, const char* what) {
  const RcclApi* R = rccl();
  const double t0 = now_s();
  long pause_ns = 100000;
  for (;;) {
    ncclResult_t st = ncclSuccess;
    ncclResult_t rc = R->CommGetAsyncError(m->c, &st);
    if (rc != ncclSuccess) st = rc;
    if (st == ncclSuccess) return 0;
    if (st != ncclInProgress) {
      R->CommAbort(m->c);
      m->c = nullptr;
      return mapa_set_error("%s: %s (rank %d of %d; communicator aborted)", what, R->GetErrorString(st), m->rank,
                            m->world);
    }
    if (now_s() - t0 > m->timeout_s) {
      R->CommAbort(m->c);
      m->c = nullptr;
      return mapa_set_error("%s: not complete after %.0f s on rank %d of %d (communicator aborted)", what,
                            m->timeout_s, m->rank, m->world);
    }
    timespec ts = {0, pause_ns};
    nanosleep(&ts, nullptr);
    pause_ns = pause_ns * 2 < 20000000 ? pause_ns * 2 : 20000000;
  }
}

static int comm_issue(mapa_comm* m, ncclResult_t rc, const char* what) {
  if (rc == ncclInProgress) return comm_wait(m, what);
  if (rc != ncclSuccess) return mapa_set_error("%s: %s (rank %d of %d)", what, rccl()->GetErrorString(rc), m->rank, m->world);
  return 0;
}

extern "C" int mapa_comm_unique_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

extern "C" int mapa_comm_get_unique_id(void* id_out) {
  MAPA_CHECK_ARG(id_out != nullptr, "mapa_comm_get_unique_id: null output");
  const RcclApi* R = rccl();
  if (!R) return -1;
  ncclUniqueId id;
  const ncclResult_t rc = R->GetUniqueId(&id);
  if (rc != ncclSuccess) return mapa_set_error("mapa_comm_get_unique_id: %s", R->GetErrorString(rc));
  memcpy(id_out, &id, sizeof(id));
  return 0;
}

extern "C" int mapa_comm_init(mapa_comm** out, int world, int rank, const void* id, int device, double timeout_s) {
  MAPA_CHECK_ARG(out && id, "mapa_comm_init: null argument");
  MAPA_CHECK_ARG(world >= 1 && rank >= 0 && rank < world, "mapa_comm_init: rank %d of %d", rank, world);
  *out = nullptr;
  const RcclApi* R = rccl();
  if (!R) return -1;
  int prev = 0;
  (void)hipGetDevice(&prev);
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return mapa_set_error("mapa_comm_init: hipSetDevice(%d): %s", device, hipGetErrorString(e));
  mapa_comm* m = new mapa_comm;
  m->world = world;
  m->rank = rank;
  m->device = device;
  m->timeout_s = timeout_s > 0 ? timeout_s : 600.0;
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclResult_t rc = R->CommInitRankConfig(&m->c, world, uid, rank, &cfg);
  int ret = 0;
  if (rc != ncclSuccess && rc != ncclInProgress) {
    if (m->c) R->CommAbort(m->c);
    ret = mapa_set_error("mapa_comm_init: ncclCommInitRankConfig: %s (rank %d of %d)", R->GetErrorString(rc), rank,
                         world);
  } else {
    ret = comm_wait(m, "mapa_comm_init");
  }
  (void)hipSetDevice(prev);
  if (ret) {
    delete m;
    return ret;
  }
  *out = m;
  return 0;
}

extern "C" int mapa_comm_allgather_kv(mapa_comm* m, void* full, int64_t slot_bytes, mapa_stream_t stream) {
  MAPA_CHECK_ARG(m && m->c && full && slot_bytes > 0, "mapa_comm_allgather_kv: bad arguments (or aborted communicator)");
  const char* mine = static_cast<const char*>(full) + (int64_t)m->rank * slot_bytes;
  return comm_issue(m, rccl()->AllGather(mine, full, (size_t)slot_bytes, ncclUint8, m->c, (hipStream_t)stream),
                    "mapa_comm_allgather_kv");
}

extern "C" int mapa_comm_broadcast(mapa_comm* m, void* buf, int64_t bytes, int root, mapa_stream_t stream) {
  MAPA_CHECK_ARG(m && m->c && buf && bytes > 0 && root >= 0 && root < m->world,
                 "mapa_comm_broadcast: bad arguments (or aborted communicator)");
  return comm_issue(m, rccl()->Broadcast(buf, buf, (size_t)bytes, ncclUint8, root, m->c, (hipStream_t)stream),
                    "mapa_comm_broadcast");
}

extern "C" int mapa_comm_check(mapa_comm* m) {
  MAPA_CHECK_ARG(m != nullptr, "mapa_comm_check: null communicator");
  if (!m->c) return mapa_set_error("mapa_comm_check: communicator aborted");
  ncclResult_t st = ncclSuccess;
  ncclResult_t rc = rccl()->CommGetAsyncError(m->c, &st);
  if (rc != ncclSuccess) st = rc;
  if (st == ncclSuccess || st == ncclInProgress) return 0;
  rccl()->CommAbort(m->c);
  m->c = nullptr;
  return mapa_set_error("mapa_comm_check: asynchronous error %s on rank %d of %d (communicator aborted)",
                        rccl()->GetErrorString(st), m->rank, m->world);
}

extern "C" int mapa_comm_destroy(mapa_comm* m, int abort) {
  if (!m) return 0;
  int ret = 0;
  if (m->c) {
    const RcclApi* R = rccl();
    if (!abort) {
      const ncclResult_t rc = R->CommFinalize(m->c);
      if (comm_issue(m, rc, "mapa_comm_destroy (finalize)") == 0 && m->c) {
        R->CommDestroy(m->c);
        m->c = nullptr;
      } else {
        ret = -1;
      }
    }
    if (m->c) R->CommAbort(m->c);
  }
  delete m;
  return ret;
}
