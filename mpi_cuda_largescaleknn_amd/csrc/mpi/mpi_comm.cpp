// Native host communicator over MPI (SURVEY §5.8 "HostComm": MPICH, host-staged).
//
// The reference is an MPI program: MPI_Init + an MPIComm wrapper (unorderedDataVariant.cu:
// 30-39, 107), ring Isend/Irecv/Waitall of device buffers (:183-193), the peer schedule's
// Allgather / Allreduce / Isend / Irecv (prePartitionedDataVariant.cu:228-229, 318-345) and
// MPI_Barrier. It relies on CUDA-aware MPI; the MPICH in this image (3.3.2, ch3:nemesis) is
// not GPU-aware, so the Python side (parallel/mpi.py) stages device tensors through pinned
// host memory and this library moves host bytes only.
//
// The pipelines' Comm interface on MPI:
//   allreduce (in place, chunked below INT_MAX elements), allgather (bytes), all-to-all-v
//   and grouped send/recv as nonblocking Isend/Irecv rounds + Waitall (messages above
//   `max_piece` bytes go in pieces: MPI counts are int), bcast, barrier, abort.
// Each call is blocking and returns 0, or non-zero with lsk_mpi_last_error() set.
#include <mpi.h>
#include <unistd.h>

#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(const char *what, int rc) {
  char msg[MPI_MAX_ERROR_STRING] = {0};
  int len = 0;
  if (rc != MPI_SUCCESS) MPI_Error_string(rc, msg, &len);
  g_err = std::string(what) + (rc != MPI_SUCCESS ? std::string(": ") + msg : std::string());
  return 1;
}

#define LSK_MPI(call)                                  \
  do {                                                 \
    const int rc_ = (call);                            \
    if (rc_ != MPI_SUCCESS) return fail(#call, rc_);   \
  } while (0)

// dtype codes shared with parallel/rccl.py (_DTYPES): 0 int8, 1 uint8, 2 int32, 4 int64,
// 7 float32, 8 float64
bool mpi_type(int code, MPI_Datatype *t, int *size) {
  switch (code) {
    case 0: *t = MPI_INT8_T; *size = 1; return true;
    case 1: *t = MPI_UINT8_T; *size = 1; return true;
    case 2: *t = MPI_INT32_T; *size = 4; return true;
    case 4: *t = MPI_INT64_T; *size = 8; return true;
    case 7: *t = MPI_FLOAT; *size = 4; return true;
    case 8: *t = MPI_DOUBLE; *size = 8; return true;
    default: return false;
  }
}

// op codes shared with parallel/rccl.py (_OPS): 0 sum, 2 max, 3 min
bool mpi_op(int code, MPI_Op *op) {
  switch (code) {
    case 0: *op = MPI_SUM; return true;
    case 2: *op = MPI_MAX; return true;
    case 3: *op = MPI_MIN; return true;
    default: return false;
  }
}

constexpr int kTag = 0x4c53;  // one tag: MPI matches same-(source, tag) messages in order

// Post the pieces of one message (Isend or Irecv) of `bytes` bytes at `p`.
int post_pieces(bool send, int peer, char *p, int64_t bytes, int64_t piece, std::vector<MPI_Request> &reqs) {
  for (int64_t off = 0; off < bytes; off += piece) {
    const int n = (int)(bytes - off < piece ? bytes - off : piece);
    MPI_Request r;
    const int rc = send ? MPI_Isend(p + off, n, MPI_BYTE, peer, kTag, MPI_COMM_WORLD, &r)
                        : MPI_Irecv(p + off, n, MPI_BYTE, peer, kTag, MPI_COMM_WORLD, &r);
    if (rc != MPI_SUCCESS) return fail(send ? "MPI_Isend" : "MPI_Irecv", rc);
    reqs.push_back(r);
  }
  return 0;
}

int64_t clamp_piece(int64_t piece) {
  if (piece <= 0 || piece > (int64_t)INT_MAX) piece = (int64_t)1 << 30;
  return piece;
}

}  // namespace

extern "C" {

const char *lsk_mpi_last_error() { return g_err.c_str(); }

int lsk_mpi_abi_version() { return 1; }

// MPI_Init_thread (SERIALIZED: collectives from the main thread, MPI_Abort from the
// watchdog thread) unless MPI is already up; returns this rank's place in COMM_WORLD.
// The watchdog thread may call lsk_mpi_abort while the main thread is inside an MPI call:
// that needs MPI_THREAD_MULTIPLE. When the library grants less (or MPI was initialised by
// someone else at a lower level), abort falls back to _exit: mpirun then tears down the
// other ranks when this one disappears (lsk_mpi_abort).
static bool g_thread_multiple = false;

int lsk_mpi_init(int *rank, int *size) {
  int inited = 0;
  LSK_MPI(MPI_Initialized(&inited));
  int provided = MPI_THREAD_SINGLE;
  if (!inited) {
    LSK_MPI(MPI_Init_thread(nullptr, nullptr, MPI_THREAD_MULTIPLE, &provided));
  } else {
    LSK_MPI(MPI_Query_thread(&provided));
  }
  g_thread_multiple = provided >= MPI_THREAD_MULTIPLE;
  // errors come back as return codes (reported through lsk_mpi_last_error), not aborts
  LSK_MPI(MPI_Comm_set_errhandler(MPI_COMM_WORLD, MPI_ERRORS_RETURN));
  LSK_MPI(MPI_Comm_rank(MPI_COMM_WORLD, rank));
  LSK_MPI(MPI_Comm_size(MPI_COMM_WORLD, size));
  return 0;
}

int lsk_mpi_finalize() {
  int inited = 0, done = 0;
  LSK_MPI(MPI_Initialized(&inited));
  LSK_MPI(MPI_Finalized(&done));
  if (inited && !done) LSK_MPI(MPI_Finalize());
  return 0;
}

// The reference's failure path: an MPI error ends the whole job (CUKD_MPI_CALL throws,
// nothing catches, mpirun tears every rank down). Here: MPI_Abort on COMM_WORLD when MPI
// allows a second thread inside it (the watchdog calls this while the main thread may be
// blocked in a collective), else _exit — the launcher ends the other ranks.
void lsk_mpi_abort(int code) {
  if (g_thread_multiple) MPI_Abort(MPI_COMM_WORLD, code);
  _exit(code ? code : 1);
}

int lsk_mpi_thread_multiple() { return g_thread_multiple ? 1 : 0; }

int lsk_mpi_barrier() {
  LSK_MPI(MPI_Barrier(MPI_COMM_WORLD));
  return 0;
}

int lsk_mpi_bcast(void *buf, int64_t bytes, int root) {
  char *p = (char *)buf;
  for (int64_t off = 0; off < bytes; off += INT_MAX) {
    const int n = (int)(bytes - off < INT_MAX ? bytes - off : INT_MAX);
    LSK_MPI(MPI_Bcast(p + off, n, MPI_BYTE, root, MPI_COMM_WORLD));
  }
  return 0;
}

int lsk_mpi_allreduce(void *buf, int64_t count, int dtype, int op) {
  MPI_Datatype t;
  MPI_Op o;
  int es = 0;
  if (!mpi_type(dtype, &t, &es)) return fail("lsk_mpi_allreduce: unsupported dtype", MPI_SUCCESS);
  if (!mpi_op(op, &o)) return fail("lsk_mpi_allreduce: unsupported op", MPI_SUCCESS);
  char *p = (char *)buf;
  for (int64_t off = 0; off < count; off += INT_MAX) {
    const int n = (int)(count - off < INT_MAX ? count - off : INT_MAX);
    LSK_MPI(MPI_Allreduce(MPI_IN_PLACE, p + off * es, n, t, o, MPI_COMM_WORLD));
  }
  return 0;
}

// recv = [size][bytes]: rank j's `bytes` bytes at recv + j * bytes.
int lsk_mpi_allgather(const void *send, void *recv, int64_t bytes, int64_t max_piece) {
  int rank = 0, size = 1;
  LSK_MPI(MPI_Comm_rank(MPI_COMM_WORLD, &rank));
  LSK_MPI(MPI_Comm_size(MPI_COMM_WORLD, &size));
  if (bytes <= (int64_t)INT_MAX) {
    LSK_MPI(MPI_Allgather(send, (int)bytes, MPI_BYTE, recv, (int)bytes, MPI_BYTE, MPI_COMM_WORLD));
    return 0;
  }
  const int64_t piece = clamp_piece(max_piece);
  std::vector<MPI_Request> reqs;
  char *r = (char *)recv;
  std::memcpy(r + (int64_t)rank * bytes, send, (size_t)bytes);
  for (int j = 0; j < size; j++) {
    if (j == rank) continue;
    if (post_pieces(false, j, r + (int64_t)j * bytes, bytes, piece, reqs)) return 1;
    if (post_pieces(true, j, (char *)send, bytes, piece, reqs)) return 1;
  }
  LSK_MPI(MPI_Waitall((int)reqs.size(), reqs.data(), MPI_STATUSES_IGNORE));
  return 0;
}

// All-to-all-v of bytes: the block at send + soff[j] (sbytes[j] bytes) goes to rank j and
// lands at recv + roff[i] on it (rbytes[i] from rank i). Self block by memcpy unless
// `force` (a forced 1-rank group then sends to itself through MPI).
int lsk_mpi_alltoallv(int size, const void *send, const int64_t *soff, const int64_t *sbytes, void *recv,
                      const int64_t *roff, const int64_t *rbytes, int64_t max_piece, int force) {
  int rank = 0, wsize = 1;
  LSK_MPI(MPI_Comm_rank(MPI_COMM_WORLD, &rank));
  LSK_MPI(MPI_Comm_size(MPI_COMM_WORLD, &wsize));
  if (size != wsize) return fail("lsk_mpi_alltoallv: size differs from MPI_COMM_WORLD", MPI_SUCCESS);
  const int64_t piece = clamp_piece(max_piece);
  std::vector<MPI_Request> reqs;
  const char *s = (const char *)send;
  char *r = (char *)recv;
  for (int j = 0; j < size; j++) {
    if (j == rank && !force) continue;
    if (rbytes[j] > 0 && post_pieces(false, j, r + roff[j], rbytes[j], piece, reqs)) return 1;
  }
  for (int j = 0; j < size; j++) {
    if (j == rank && !force) {
      if (sbytes[j] != rbytes[j]) return fail("lsk_mpi_alltoallv: self block sizes differ", MPI_SUCCESS);
      if (sbytes[j] > 0) std::memcpy(r + roff[j], s + soff[j], (size_t)sbytes[j]);
      continue;
    }
    if (sbytes[j] > 0 && post_pieces(true, j, (char *)s + soff[j], sbytes[j], piece, reqs)) return 1;
  }
  if (!reqs.empty()) LSK_MPI(MPI_Waitall((int)reqs.size(), reqs.data(), MPI_STATUSES_IGNORE));
  return 0;
}

// Grouped point-to-point (the reference's Isend/Irecv/Waitall rounds): ns sends of
// sbytes[i] at sbuf[i] to dst[i], nr receives of rbytes[i] into rbuf[i] from src[i].
int lsk_mpi_sendrecv(int ns, const int *dst, void *const *sbuf, const int64_t *sbytes, int nr, const int *src,
                     void *const *rbuf, const int64_t *rbytes, int64_t max_piece) {
  const int64_t piece = clamp_piece(max_piece);
  std::vector<MPI_Request> reqs;
  for (int i = 0; i < nr; i++)
    if (rbytes[i] > 0 && post_pieces(false, src[i], (char *)rbuf[i], rbytes[i], piece, reqs)) return 1;
  for (int i = 0; i < ns; i++)
    if (sbytes[i] > 0 && post_pieces(true, dst[i], (char *)sbuf[i], sbytes[i], piece, reqs)) return 1;
  if (!reqs.empty()) LSK_MPI(MPI_Waitall((int)reqs.size(), reqs.data(), MPI_STATUSES_IGNORE));
  return 0;
}

}  // extern "C"
