// Native RCCL communicator (SURVEY §5.8 RcclComm): the reference calls CUDA-aware MPI from
// C++ (MPIComm + CUKD_MPI_CALL, unorderedDataVariant.cu:23-39; Isend/Irecv ring
// :183-193, Allreduce/Allgather/Barrier call sites in SURVEY §2.6). Here the collectives
// of the k-NN exchange go straight to RCCL (xGMI peer-to-peer on an MI355X node) on the
// caller's HIP stream — no process-group wrapper, no internal stream hop — so an
// exchange issued on the pipeline's high-priority side stream runs under the k-NN.
//
// RCCL is opened at run time (dlopen of an explicit path, RTLD_LOCAL, symbols via dlsym):
// torch ships its own librccl.so.1 (2.26) with the same SONAME, and binding by path keeps
// the two instances apart (the caller picks which one: ROCm's 2.27 by default).
//
// Large messages: every point-to-point message is cut into pieces of at most `piece`
// bytes; round r carries piece r of every pair inside one ncclGroupStart/End (both ends
// know each message size, so pieces pair up in posting order). RCCL 2.26 corrupts single
// messages above 1 GiB (profiles/r2_rccl); pieces keep every version below that.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {

thread_local std::string g_err;

struct Api {
  void *h = nullptr;
  decltype(&ncclGetVersion) getVersion = nullptr;
  decltype(&ncclGetUniqueId) getUniqueId = nullptr;
  decltype(&ncclCommInitRank) commInitRank = nullptr;
  decltype(&ncclCommDestroy) commDestroy = nullptr;
  decltype(&ncclCommAbort) commAbort = nullptr;
  decltype(&ncclCommGetAsyncError) asyncError = nullptr;
  decltype(&ncclGetErrorString) errorString = nullptr;
  decltype(&ncclAllReduce) allReduce = nullptr;
  decltype(&ncclAllGather) allGather = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) groupStart = nullptr;
  decltype(&ncclGroupEnd) groupEnd = nullptr;
};
Api g_api;

int fail(const std::string &m) {
  g_err = m;
  return 1;
}

int nccl_fail(const char *what, ncclResult_t r) {
  const char *s = g_api.errorString ? g_api.errorString(r) : "?";
  return fail(std::string(what) + ": " + s + " (" + std::to_string((int)r) + ")");
}

#define LSK_NCCL(call, what)                         \
  do {                                               \
    ncclResult_t r_ = (call);                        \
    if (r_ != ncclSuccess) return nccl_fail(what, r_); \
  } while (0)

template <class F>
bool sym(void *h, const char *name, F &out) {
  out = reinterpret_cast<F>(dlsym(h, name));
  return out != nullptr;
}

int need_api() { return g_api.h ? 0 : fail("RCCL not loaded (lsk_comm_load)"); }

// grouped send/recv rounds over contiguous byte ranges
struct Msg {
  int peer;
  char *buf;
  int64_t bytes;
};

int rounds(ncclComm_t comm, const std::vector<Msg> &sends, const std::vector<Msg> &recvs, int64_t piece,
           hipStream_t st) {
  piece = std::max<int64_t>(piece, 1);
  int64_t nr = 0;
  for (const Msg &m : sends) nr = std::max(nr, (m.bytes + piece - 1) / piece);
  for (const Msg &m : recvs) nr = std::max(nr, (m.bytes + piece - 1) / piece);
  for (int64_t r = 0; r < nr; r++) {
    LSK_NCCL(g_api.groupStart(), "ncclGroupStart");
    for (const Msg &m : sends) {
      const int64_t o = r * piece;
      if (o < m.bytes)
        LSK_NCCL(g_api.send(m.buf + o, (size_t)std::min(piece, m.bytes - o), ncclUint8, m.peer, comm, st),
                 "ncclSend");
    }
    for (const Msg &m : recvs) {
      const int64_t o = r * piece;
      if (o < m.bytes)
        LSK_NCCL(g_api.recv(m.buf + o, (size_t)std::min(piece, m.bytes - o), ncclUint8, m.peer, comm, st),
                 "ncclRecv");
    }
    LSK_NCCL(g_api.groupEnd(), "ncclGroupEnd");
  }
  return 0;
}

}  // namespace

extern "C" {

const char *lsk_comm_last_error() { return g_err.c_str(); }

// Load RCCL from `path` (once per process; a second call with any path is a no-op).
int lsk_comm_load(const char *path) {
  if (g_api.h) return 0;
  void *h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return fail(std::string("dlopen ") + path + ": " + dlerror());
  Api a;
  a.h = h;
  const bool ok = sym(h, "ncclGetVersion", a.getVersion) && sym(h, "ncclGetUniqueId", a.getUniqueId) &&
                  sym(h, "ncclCommInitRank", a.commInitRank) && sym(h, "ncclCommDestroy", a.commDestroy) &&
                  sym(h, "ncclCommAbort", a.commAbort) && sym(h, "ncclGetErrorString", a.errorString) &&
                  sym(h, "ncclCommGetAsyncError", a.asyncError) &&
                  sym(h, "ncclAllReduce", a.allReduce) && sym(h, "ncclAllGather", a.allGather) &&
                  sym(h, "ncclSend", a.send) && sym(h, "ncclRecv", a.recv) &&
                  sym(h, "ncclGroupStart", a.groupStart) && sym(h, "ncclGroupEnd", a.groupEnd);
  if (!ok) {
    dlclose(h);
    return fail(std::string(path) + ": missing RCCL symbols");
  }
  g_api = a;
  return 0;
}

int lsk_comm_version(int *v) {
  if (need_api()) return 1;
  LSK_NCCL(g_api.getVersion(v), "ncclGetVersion");
  return 0;
}

int lsk_comm_unique_id(unsigned char *out, int cap) {
  if (need_api()) return 1;
  if (cap < (int)sizeof(ncclUniqueId)) return fail("unique id buffer too small");
  ncclUniqueId id;
  LSK_NCCL(g_api.getUniqueId(&id), "ncclGetUniqueId");
  std::memcpy(out, &id, sizeof(id));
  return (int)sizeof(id) == NCCL_UNIQUE_ID_BYTES ? 0 : fail("unexpected ncclUniqueId size");
}

int lsk_comm_id_bytes() { return NCCL_UNIQUE_ID_BYTES; }

int lsk_comm_init(const unsigned char *idb, int nranks, int rank, int device, void **out) {
  if (need_api()) return 1;
  if (hipSetDevice(device) != hipSuccess) return fail("hipSetDevice failed");
  ncclUniqueId id;
  std::memcpy(&id, idb, sizeof(id));
  ncclComm_t c = nullptr;
  LSK_NCCL(g_api.commInitRank(&c, nranks, id, rank), "ncclCommInitRank");
  *out = c;
  return 0;
}

int lsk_comm_destroy(void *comm, int abort) {
  if (need_api() || !comm) return 1;
  if (abort) {
    LSK_NCCL(g_api.commAbort((ncclComm_t)comm), "ncclCommAbort");
  } else {
    LSK_NCCL(g_api.commDestroy((ncclComm_t)comm), "ncclCommDestroy");
  }
  return 0;
}

// Asynchronous communicator error (a peer died, a network/xGMI failure): polled by the
// watchdog thread (ncclCommGetAsyncError is thread-safe); *msg gets RCCL's error string.
int lsk_comm_async_error(void *comm, int *err, const char **msg) {
  if (need_api() || !comm) return 1;
  ncclResult_t r = ncclSuccess;
  LSK_NCCL(g_api.asyncError((ncclComm_t)comm, &r), "ncclCommGetAsyncError");
  *err = (int)r;
  *msg = g_api.errorString(r);
  return 0;
}

// dtype / op: ncclDataType_t / ncclRedOp_t values (rccl.h), passed through
int lsk_comm_allreduce(void *comm, void *buf, int64_t count, int dtype, int op, void *stream) {
  if (need_api()) return 1;
  LSK_NCCL(g_api.allReduce(buf, buf, (size_t)count, (ncclDataType_t)dtype, (ncclRedOp_t)op, (ncclComm_t)comm,
                           (hipStream_t)stream),
           "ncclAllReduce");
  return 0;
}

int lsk_comm_allgather(void *comm, const void *send, void *recv, int64_t bytes, void *stream) {
  if (need_api()) return 1;
  LSK_NCCL(g_api.allGather(send, recv, (size_t)bytes, ncclUint8, (ncclComm_t)comm, (hipStream_t)stream),
           "ncclAllGather");
  return 0;
}

// all-to-all-v of byte ranges: send[soff[j], +sbytes[j]) -> rank j, recv[roff[j], +rbytes[j])
// <- rank j. The own-rank pair is a device copy unless `self_rccl` (forced 1-rank tests:
// RCCL carries it too).
int lsk_comm_alltoallv(void *comm, int nranks, int rank, const void *send, const int64_t *soff,
                       const int64_t *sbytes, void *recv, const int64_t *roff, const int64_t *rbytes, int64_t piece,
                       int self_rccl, void *stream) {
  if (need_api()) return 1;
  hipStream_t st = (hipStream_t)stream;
  std::vector<Msg> s, r;
  for (int j = 0; j < nranks; j++) {
    if (j == rank && !self_rccl) {
      if (sbytes[j] != rbytes[j]) return fail("alltoallv: own-rank send and receive sizes differ");
      if (sbytes[j] > 0 &&
          hipMemcpyAsync((char *)recv + roff[j], (const char *)send + soff[j], (size_t)sbytes[j],
                         hipMemcpyDeviceToDevice, st) != hipSuccess)
        return fail("alltoallv: own-rank copy failed");
      continue;
    }
    if (sbytes[j] > 0) s.push_back({j, (char *)send + soff[j], sbytes[j]});
    if (rbytes[j] > 0) r.push_back({j, (char *)recv + roff[j], rbytes[j]});
  }
  return rounds((ncclComm_t)comm, s, r, piece, st);
}

// grouped point-to-point: nsend messages (peer, buffer, bytes) out, nrecv in
int lsk_comm_sendrecv(void *comm, int nsend, const int *speer, void *const *sbuf, const int64_t *sbytes, int nrecv,
                      const int *rpeer, void *const *rbuf, const int64_t *rbytes, int64_t piece, void *stream) {
  if (need_api()) return 1;
  std::vector<Msg> s, r;
  for (int i = 0; i < nsend; i++)
    if (sbytes[i] > 0) s.push_back({speer[i], (char *)sbuf[i], sbytes[i]});
  for (int i = 0; i < nrecv; i++)
    if (rbytes[i] > 0) r.push_back({rpeer[i], (char *)rbuf[i], rbytes[i]});
  return rounds((ncclComm_t)comm, s, r, piece, (hipStream_t)stream);
}

}  // extern "C"
