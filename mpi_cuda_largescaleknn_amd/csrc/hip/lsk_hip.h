// lsknn gfx950 kernel library — C ABI (ctypes from Python; the caller owns all memory).
//
// Every entry point takes the HIP stream to launch on (torch's current stream when
// called from Python) and never allocates, synchronises or copies to the host, so a
// whole local pipeline can be captured into a hipGraph. Workspace sizes come from the
// *_ws_bytes queries. Return value: 0 on success, a hipError_t otherwise
// (lsk_hip_last_error() has the message).
//
// Layout conventions
//   points   : packed float3 (12 B) arrays; arrays read by the k-NN kernel must carry
//              64 points of readable padding after the last point (scalar loads fetch
//              candidates in 8-point chunks).
//   tree     : implicit complete binary tree over 64-point Morton buckets. Node i
//              (root = 1) is two float4: lo.xyz + lo.w = max squared k-NN radius of the
//              queries below it (halo publishing), hi.xyz + hi.w unused. Leaves are at
//              level `depth`: node (1<<depth)+b covers sorted points [64b, 64b+64).
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int lsk_hip_abi_version(void);
// Uniform-density estimate of the k-th squared distance from a bounds box [8] and the
// global point count, written to out[0] on the device (= knn_engine.radius_hint2).
int lsk_hip_radius_hint(const float *box, int64_t n_total, int32_t k, float *out, void *stream);
const char *lsk_hip_last_error(void);
int lsk_hip_device_info(int device, char *buf, int buflen);

// ---- bounds / Morton / permutation helpers ---------------------------------------
size_t lsk_hip_bounds_ws_bytes(int64_t n);
// box_out: 8 floats on device: lo.xyz, hi.xyz, cube scale (1024/extent), extent.
int lsk_hip_bounds(const float *pts, int64_t n, float *box_out, void *ws, void *stream);
// Recompute box_out[6..7] from box_out[0..5] (after a cross-rank min/max reduction).
int lsk_hip_box_finalize(float *box, void *stream);
// keys[i] = 30-bit space-filling-curve key of pts[i] in the cube of `box` (curve:
// 0 = Morton, 1 = Hilbert, common.h); vals[i] = i (if vals is not null).
int lsk_hip_morton(const float *pts, int64_t n, const float *box, uint32_t *keys,
                   uint32_t *vals, int curve, void *stream);
// same with vals[i] = base + i and an optional device flag (nothing happens if *flag == 0)
int lsk_hip_morton_ex(const float *pts, int64_t n, const float *box, uint32_t *keys, uint32_t *vals, int curve,
                      int64_t base, const int *flag, void *stream);
// dst[i] = src[idx[i]] (float3 gather).
int lsk_hip_gather3(const float *src, const uint32_t *idx, int64_t n, float *dst, void *stream);
// dst[idx[i]] = src[i] (float scatter), optional sqrt-finalisation.
int lsk_hip_scatter1(const float *src, const uint32_t *idx, int64_t n, float *dst,
                     int finalize_sqrt, void *stream);
// out[i] = finalize(src[i]) (sqrt unless inf).
int lsk_hip_finalize(const float *src, int64_t n, float *dst, void *stream);
// keys[i] = destination rank of point i: number of splitters s with (morton>>shift) >= s.
int lsk_hip_dest_rank(const uint32_t *morton, int64_t n, const uint32_t *splitters,
                      int nsplit, int shift, uint32_t *dest, uint32_t *vals, void *stream);
// hist[key >> shift] += 1 over every `sample`-th key (hist: uint32 of size
// 1<<(30-shift), zeroed by caller).
int lsk_hip_key_histogram(const uint32_t *keys, int64_t n, int shift, int sample, uint32_t *hist,
                          void *stream);
// counts[dest[i]] += 1 for dest < ndest (counts zeroed by caller).
int lsk_hip_count_dest(const uint32_t *dest, int64_t n, int ndest, uint32_t *counts,
                       void *stream);

// Bounding boxes of contiguous segments: seg[i] (non-decreasing runs) = segment of point
// i; lo/hi: [nseg][3] floats (overwritten). Wave reductions + one atomic per segment and
// wave (no contended per-point atomics).
int lsk_hip_segment_bounds(const float *pts, const uint32_t *seg, int64_t m, int64_t nseg,
                           float *lo, float *hi, void *stream);

// ---- LSD radix sort of (uint32 key, uint32 value) pairs ------------------------------
size_t lsk_hip_sort_ws_bytes(int64_t n);
// Sorts by key bits [0, key_bits). Uses keys_alt/vals_alt as ping-pong buffers;
// *result_in_alt is set to 1 if the sorted output ended in the alt buffers.
int lsk_hip_sort_pairs(uint32_t *keys, uint32_t *vals, uint32_t *keys_alt, uint32_t *vals_alt,
                       int64_t n, int key_bits, void *ws, int *result_in_alt, void *stream);

// ---- bucket tree ---------------------------------------------------------------------
int lsk_hip_tree_depth(int64_t n);          // depth for 64-point buckets
int64_t lsk_hip_tree_nodes(int64_t n);      // number of node slots (2^(depth+1))
// qnodes (optional, 2^depth*4 x 2 float4): boxes of the four 16-point quarters of
// every bucket (quarter q of bucket b = sorted points [64b+16q, 64b+16q+16)).
int lsk_hip_build_tree(const float *sorted_pts, int64_t n, float *nodes, float *qnodes,
                       void *stream);
// leaves' lo.w = max over the bucket's queries of d2[i]; propagated to all levels.
int lsk_hip_tree_set_radii(float *nodes, int64_t n, const float *d2_sorted, void *stream);
// a-priori upper bound of each node's k-th squared radius (from the sorted points and
// bucket boxes only, before any query ran)
int lsk_hip_tree_set_radii_ub(float *nodes, const float *sorted_pts, int64_t n, int k, void *stream);

// ---- k-th-distance selection ----------------------------------------------------------
typedef struct lsk_tree_view {
  const float *pts;    // sorted points (padded)
  const float *nodes;  // node array
  const float *qnodes; // quarter boxes (row kernel)
  int64_t n;
  int32_t depth;
  int32_t pad;
} lsk_tree_view;

typedef struct lsk_knn_args {
  const float *qpts;        // sorted query points; groups of 64 consecutive queries
  int64_t nq;
  const uint32_t *groups;   // optional list of query groups to (re)process
  int64_t ngroups;          // length of `groups` (ignored when groups == NULL)
  lsk_tree_view tree[2];
  int32_t ntrees;
  int32_t k;
  float cut2;               // (-r R)^2 as float; +inf by default
  float r_hint2;            // global estimate of the k-th squared distance; < 0: read it
                            // from tree[0].nodes[3] (the unused node 0, where
                            // lsk_hip_radius_hint's value was copied: no host round trip)
  float *out_d2;            // [nq] k-th squared distance per query (sorted order), or NULL
  unsigned long long *stats;  // optional [16] 64-bit counters (NULL = off)
  uint32_t *qstatus;        // optional [nq] per-query status bits (NULL = off)
  int32_t seed;             // queries are tree[0]'s points: seed pass 1 with buckets
                            // [g-seed, g+seed] of tree 0 (0 = off)
  int32_t pad0;
  const float *init_d2;     // optional [nq] known upper bound of each query's k-th squared
                            // distance (a re-query after a halo exchange passes the local
                            // result): the first range ends just above it (NULL = estimate)
  const uint32_t *out_perm; // optional fused result scatter: when set, the kernel also
  float *out_final;         // writes out_final[out_perm[q]] = sqrtf(d2) (inf stays inf),
                            // which saves a separate scatter kernel
  uint32_t *fail_list;      // failure list of the 16-bit kernel (knn_rows): sorted-order
  uint32_t *fail_count;     // query indices it could not resolve exactly, and their count
  int64_t fail_cap;         // (the count may exceed the capacity: then the host reruns all)
  int32_t debug_fail_mod;   // tests only: also fail every query qi with qi % mod == 0
  int32_t pad1;
  const int32_t *gate;      // optional device flag (lsk_hip_grid_decide): the rows / grid
  int32_t gate_on;          // kernel runs only when *gate == gate_on (else every wave
  int32_t pad2;             // returns at once): both are queued, the device picks one
  const uint32_t *ngroups_dev;  // optional, with `groups`: the list's length on the device
                                // (ngroups is then the launch's upper bound; no host read)
} lsk_knn_args;

// Production kernel: 4 x 16-query rows, 16-bit LDS histogram radix select. Queries it
// cannot resolve exactly (bin overflow, pass limit, collect mismatch, walk guard) get a
// NaN placeholder and are appended to fail_list (fail_count is the always-on failure word).
int lsk_hip_knn_rows(const lsk_knn_args *args, void *stream);
// Exact backstop for any input and any k >= 1: wave per query, 32-bit bins. list != NULL:
// the queries list[0 .. min(*count, cap)) (count is read on the device: graph-capturable,
// an empty list costs one short launch); list == NULL: every query (or every query of
// args->groups).
int lsk_hip_knn_exact(const lsk_knn_args *args, const uint32_t *list, const uint32_t *count,
                      int64_t cap, void *stream);

// ---- cell-grid candidate source (knn_grid.hip) -----------------------------------------
// Octree grid over the curve-sorted points of one tree (cube = the sort keys' box): every
// cell of level `level` has 64 slots, one per grandchild (level + 2 <= 10) in curve order
// (= memory order), each the grandchild's contiguous run of the sorted array:
// (start, end, x | y << 10 | z << 20, 0) as uint32 x 4; empty: (0, 0, ...). Cells are
// indexed by the Morton code of their coordinates.
typedef struct lsk_grid_view {
  const uint32_t *slots;  // [8^level * 64][4]
  const uint32_t *pad_;   // (unused)
  const float *box;       // [8] device: the box of the sort keys (lo.xyz, hi.xyz, scale, extent)
  const float *inf4;      // [4] device: +inf (unused padding source)
  int32_t level;
  int32_t pad;
} lsk_grid_view;
int lsk_hip_grid_build(const float *sorted_pts, const uint32_t *sorted_keys, int64_t n, const float *box,
                       int32_t level, uint32_t *slots, void *stream);
// counts[l] (l = 1..10, 11 slots, zeroed here) = number of adjacent sorted keys whose level-l
// prefixes differ (distinct level-l cells = counts[l] + 1).
int lsk_hip_key_levels(const uint32_t *keys, int64_t n, unsigned long long *counts, void *stream);
// out[0] = sum over slots of population^2 (zeroed here).
int lsk_hip_grid_sq(const uint32_t *slots, int64_t nslot, unsigned long long *out, void *stream);
// Device-side "does the grid apply" (no host read, graph-capturable): gate[0] = 1 iff the
// level census (counts: lsk_hip_key_levels) says near-uniform 3-D data at grandchild level
// g — occupied cells multiply by >= 6 from g-1 to g and their mean population is in
// [2, 256] — and the mean population of a point's own grandchild (sq: lsk_hip_grid_sq /
// n) is at most crowd * (mean + 1); check == 0: gate[0] = 1 unconditionally.
int lsk_hip_grid_decide(const unsigned long long *counts, const unsigned long long *sq, int64_t n, int32_t g,
                        float crowd, int32_t check, int32_t *gate, void *stream);
// Near-uniform fast path of lsk_hip_knn_rows (same contract, same failure list): one tree
// whose points are the queries, no groups / init_d2; candidates from the grid.
int lsk_hip_knn_grid(const lsk_knn_args *args, const lsk_grid_view *grid, void *stream);

// ---- halo exchange -------------------------------------------------------------------
// Published tree: the top `levels` levels of a tree (node slots 1 .. 2^levels-1... up to
// 2^(levels+1)), each node 8 floats (lo.xyz, r2, hi.xyz, pad).
// mask[i] bit j set iff point i must be sent to rank j (j != self).
// Boundary classification of the local query groups before the local pass: flags[g] = 1
// iff the box of local bucket g (leaf of local_nodes, depth `depth`), inflated by its
// squared radius bound lo.w, comes strictly closer than that bound to some node of
// another rank's published tree — i.e. some other rank's point could be among the k
// nearest of one of the group's queries. flags[g] = 0 groups need no halo at all.
int lsk_hip_boundary_groups(const float *local_nodes, int32_t depth, int64_t ngroups, const float *pub,
                            const int64_t *pub_off, const int32_t *pub_depth, int nranks, int self,
                            uint32_t *flags, void *stream);
int lsk_hip_halo_mask(const float *pts, int64_t n, const float *pub, const int64_t *pub_off,
                      const int32_t *pub_depth, int nranks, int self, uint64_t *mask,
                      void *stream);
// Flag query groups (64 consecutive sorted queries) that may have a closer halo point:
// flags[g] = 1 iff some halo leaf box is strictly closer to one of the group's queries
// than that query's current k-th squared distance qd2.
int lsk_hip_flag_query_groups(const float *qpts, const float *qd2, int64_t nq,
                              const float *halo_nodes, int32_t halo_depth, int64_t nhalo,
                              uint32_t *flags, void *stream);
// Compacts indices i with flags[i] != 0 into list; *count (device) receives the count.
// Same purpose, exact-superset and independent of the halo tree's boxes: every halo
// point walks the local radius-annotated tree (tree_set_radii) and sets flags[g] = 1 for
// each bucket g whose inflated box contains it. flags must be zeroed by the caller.
int lsk_hip_flag_groups_inverse(const float *halo_pts, int64_t nh, const float *local_nodes,
                                int32_t depth, int64_t ngroups, uint32_t *flags, void *stream);
int lsk_hip_compact_flags(const uint32_t *flags, int64_t n, uint32_t *list, uint32_t *count,
                          void *stream);
// For each destination rank j: writes the points with mask bit j into send buffer at
// offsets[j] + (running cursor). cursors: device [nranks] zeroed by caller.
int lsk_hip_halo_pack(const float *pts, const uint64_t *mask, int64_t n, int nranks,
                      const int64_t *offsets, uint32_t *cursors, float *send, void *stream);
int lsk_hip_mask_counts(const uint64_t *mask, int64_t n, int nranks, uint32_t *counts,
                        void *stream);

// ---- ref-algo (reference algorithm baseline, refalgo.hip) -----------------------------
// Sortable bits of coord[dim] -> keys, iota -> vals.
int lsk_hip_lbt_keys(const float *pts, int64_t n, int dim, uint32_t *keys, uint32_t *vals,
                     void *stream);
// Tag update of the left-balanced builder for `level` (points sorted by (tag, coord)).
int lsk_hip_lbt_retag(uint32_t *tags, int64_t n, int level, void *stream);
int lsk_hip_gather_u32(const uint32_t *src, const uint32_t *idx, int64_t n, uint32_t *dst,
                       void *stream);
// runQuery: stack-free traversal of a left-balanced tree, global AoS k-max-heaps.
int lsk_hip_refalgo_knn(const float *tree, int64_t n, const float *qpts, int64_t nq,
                        unsigned long long *heaps, int k, float cut2, int init, float *rmax,
                        uint32_t id_base, void *stream);
// extractFinalResult
int lsk_hip_refalgo_extract(const unsigned long long *heaps, int64_t nq, int k, float *out,
                            void *stream);

// ---- verification (verify.hip) --------------------------------------------------------
// counts[2j] += #{p : dist2(q_j, p) < thr[2j]}, counts[2j+1] += #{p : dist2(q_j, p) < thr[2j+1]}
// over the n points (nq <= 1024 queries; counts zeroed by the caller, accumulated).
int lsk_hip_count_below(const float *pts, int64_t n, const float *q, const float *thr, int nq,
                        unsigned long long *counts, void *stream);

#ifdef __cplusplus
}
#endif
