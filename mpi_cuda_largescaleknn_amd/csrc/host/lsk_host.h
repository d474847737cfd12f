// lsknn host library — C ABI (loaded from Python with ctypes; usable from C++ apps).
//
// Components (SURVEY §2 IDs):
//   A01/A02/A03  CLI grammar of both reference entrypoints        -> lsk_cli_parse
//   A06          readFilePortion<float3> partition semantics       -> lsk_io_portion / lsk_io_read
//   A07          readListOfFileNames (fixed: CRLF, no trailing \n)  -> lsk_io_read_filelist
//   A22/A23      output writers (parallel pwrite, same bytes)      -> lsk_io_write
//   A18-A21      prePartitioned peer schedule                      -> lsk_peer_*
//   T1 oracle    exact CPU k-th-distance (brute force / k-d tree)  -> lsk_cpu_kth_*
//   CPU backend  Morton keys, bounds, halo filter for gloo tests   -> lsk_cpu_*
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// ---------------------------------------------------------------- version / info
int lsk_host_abi_version(void);

// ---------------------------------------------------------------- CLI (A01-A03, C7)
// variant: 0 = unorderedData, 1 = prePartitionedData.
// Returns 0 on success; otherwise the exit code usage() would use (1) and writes the
// complete stderr text the reference prints into `err` (NUL-terminated, truncated to
// errlen). Extension flags (all long options, defaults never change reference
// behaviour) are parsed into the same struct.
typedef struct lsk_cli_args {
  char input[4096];   // positional (last wins)
  char output[4096];  // -o
  int k;              // -k
  float max_radius;   // -r  (default +inf)
  int gpu_affinity;   // -g  (0 = unset)
  // extensions
  char mode[32];      // --mode {auto,halo,ring,peer}
  char device[16];    // --device {auto,cuda,cpu}
  char stats[4096];   // --stats <file.json>
  int verbose;        // -v / --verbose
  char bootstrap[16]; // --bootstrap {auto,env,mpi,spawn}: where rank/size come from
  int nproc;          // --nproc N: ranks started by --bootstrap spawn (0 = unset)
  char device_map[256];  // --device-map 0,1,...: local rank i uses GPU map[i % len]
  char balance[8];    // --balance {auto,on,off}: prePartitioned load rebalancing
} lsk_cli_args;

int lsk_cli_parse(int variant, int argc, const char **argv, lsk_cli_args *out, char *err,
                  int errlen);

// ---------------------------------------------------------------- I/O (A06, A07, A22/A23)
// Reference partition: numData = bytes/recsize, rank r of P gets
// [floor(numData*r/P), floor(numData*(r+1)/P)). Returns 0 or -errno.
int lsk_io_portion(const char *path, int64_t rank, int64_t size, int64_t recsize,
                   int64_t *begin, int64_t *count, int64_t *total);
// Multi-threaded pread of nbytes at offset into dst. Returns 0 or -errno.
int lsk_io_read(const char *path, int64_t offset, int64_t nbytes, void *dst, int nthreads);
// Multi-threaded pwrite. flags bit0: create+truncate first, bit1: ftruncate to
// `total_size` (when >= 0) before writing. Returns 0 or -errno.
int lsk_io_write(const char *path, int64_t offset, const void *src, int64_t nbytes,
                 int flags, int64_t total_size, int nthreads);
// Reads a file list. Writes names separated by '\n' into buf; returns the number of
// names, or -errno, or -(needed bytes) - 1000000 if buf is too small.
int64_t lsk_io_read_filelist(const char *path, char *buf, int64_t buflen);

// ---------------------------------------------------------------- peer schedule (A18-A21)
// Sattolo permutation seeded exactly like the reference (srand(rank+0x1234567), 10
// discarded rand() calls). Writes `size` ints.
void lsk_peer_permutation(int rank, int size, int *out);
// boxes: 6 floats per rank (lo.xyz, hi.xyz). seen: one byte per rank. Returns the
// requested peer or -1 (strictly closest by box gap among unseen peers with gap <
// cutoff; ties go to the first in permutation order).
int lsk_peer_choose(const float *my_box, const float *all_boxes, int size, float cutoff,
                    const uint8_t *seen, const int *perm);
float lsk_box_distance(const float *a, const float *b);

// ---------------------------------------------------------------- CPU oracle (T1)
// Result semantics: for every query, the k-th smallest of the multiset
// { dist2(q,p) : p in points, dist2 < cut2 } ∪ { cut2 repeated k }, as a squared
// distance. cut2 = r*r (float) or +inf.
void lsk_cpu_kth_brute(const float *pts, int64_t n, const float *qry, int64_t nq, int k,
                       float cut2, float *out_d2, int nthreads);
// Verification counts (= lsk_hip_count_below): counts[2j] += #{p : dist2(q_j,p) < thr[2j]},
// counts[2j+1] += #{p : dist2(q_j,p) < thr[2j+1]}.
void lsk_cpu_count_below(const float *pts, int64_t n, const float *qry, const float *thr, int nq,
                         unsigned long long *counts, int nthreads);
// Same result via a CPU k-d tree (object-median, leaf buckets) built over `pts`.
void lsk_cpu_kth_kdtree(const float *pts, int64_t n, const float *qry, int64_t nq, int k,
                        float cut2, float *out_d2, int nthreads);

// ---------------------------------------------------------------- CPU backend ops
// AABB of n points -> box[6]. Empty set -> (+inf,-inf).
void lsk_cpu_bounds(const float *pts, int64_t n, float *box, int nthreads);
// 30-bit curve keys (curve: 0 = Morton, 1 = Hilbert) relative to a cube (origin,
// scale = 1024/extent).
void lsk_cpu_morton(const float *pts, int64_t n, const float *origin, float scale,
                    uint32_t *keys, int curve, int nthreads);
// For each point, the bitmask (bit j) of target sets it must be sent to: point p goes
// to set j iff box_dist2(p, box) < r2 for some box of set j. boxes: 8 floats each
// (lo.xyz, r2, hi.xyz, pad); box_offsets: nsets+1 offsets. skip_set excluded (-1 none).
void lsk_cpu_halo_mask(const float *pts, int64_t n, const float *boxes,
                       const int64_t *box_offsets, int nsets, int skip_set,
                       uint64_t *mask, int nthreads);

// ---------------------------------------------------------------- ref-algo (CPU twin)
// Left-balanced k-d tree (object median, round-robin axis): out_pts in tree order,
// out_ids[i] = input index of tree node i (may be NULL).
void lsk_cpu_lbt_build(const float *pts, int64_t n, float *out_pts, uint32_t *out_ids);
// Stack-free traversal + persisted k-max-heaps (AoS [nq][k] of d2bits<<32|id); init=1
// (re)initialises with cut2; rmax (optional) receives max(rmax, max_q sqrt(top_q)).
void lsk_cpu_refalgo_knn(const float *tree, int64_t n, const float *qpts, int64_t nq,
                         unsigned long long *heaps, int k, float cut2, int init, float *rmax,
                         uint32_t id_base, int nthreads);
void lsk_cpu_refalgo_extract(const unsigned long long *heaps, int64_t nq, int k, float *out);

#ifdef __cplusplus
}
#endif
