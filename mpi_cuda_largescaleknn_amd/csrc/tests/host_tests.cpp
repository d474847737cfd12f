// Host unit tests (SURVEY §4.2 tier T0), CTest target `host_tests`.
//
// Covers the reference's observable host behaviour re-implemented in liblsknn_host:
//   * readFilePortion partition math (unorderedDataVariant.cu:42-63): floor(n*r/P)
//     ranges, trailing partial records ignored;
//   * file list parsing (prePartitionedDataVariant.cu:114-126) with the documented fixes
//     (CRLF stripped, unterminated last line kept);
//   * CLI grammar and error texts (unorderedDataVariant.cu:66-71, 114-135);
//   * the Sattolo peer permutation (prePartitionedDataVariant.cu:136-148), the box gap
//     (:150-155) and the peer choice (:157-174);
//   * the two CPU oracles agree (brute force vs k-d tree) including -r semantics.
// No GPU needed. Exit status 0 = all passed.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <random>
#include <string>
#include <vector>

#include "lsk_host.h"

static int g_fail = 0;
#define CHECK(cond)                                                   \
  do {                                                                \
    if (!(cond)) {                                                    \
      fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      g_fail++;                                                       \
    }                                                                 \
  } while (0)

static std::string tmpfile_with(const void *data, size_t n) {
  char path[] = "/tmp/lsknn_host_test_XXXXXX";
  int fd = mkstemp(path);
  if (fd < 0) abort();
  if (n && write(fd, data, n) != (ssize_t)n) abort();
  close(fd);
  return path;
}

static void test_partition() {
  // 10 records + 5 trailing bytes; P = 3 -> [0,3) [3,6) [6,10)
  std::vector<char> bytes(10 * 12 + 5, 7);
  std::string p = tmpfile_with(bytes.data(), bytes.size());
  int64_t b, c, t;
  const int64_t want_b[3] = {0, 3, 6}, want_c[3] = {3, 3, 4};
  for (int r = 0; r < 3; r++) {
    CHECK(lsk_io_portion(p.c_str(), r, 3, 12, &b, &c, &t) == 0);
    CHECK(b == want_b[r] && c == want_c[r] && t == 10);
  }
  // more ranks than records: some ranks get nothing, ranges still tile [0, n)
  int64_t next = 0;
  for (int r = 0; r < 16; r++) {
    CHECK(lsk_io_portion(p.c_str(), r, 16, 12, &b, &c, &t) == 0);
    CHECK(b == next);
    next = b + c;
  }
  CHECK(next == 10);
  CHECK(lsk_io_portion("/nonexistent/file", 0, 1, 12, &b, &c, &t) < 0);
  unlink(p.c_str());
}

static void test_read_write_roundtrip() {
  std::vector<float> v(3 * 1000);
  for (size_t i = 0; i < v.size(); i++) v[i] = (float)i * 0.5f;
  std::string p = tmpfile_with(nullptr, 0);
  CHECK(lsk_io_write(p.c_str(), 0, v.data(), (int64_t)(v.size() * 4), 1, -1, 4) == 0);
  std::vector<float> w(v.size());
  CHECK(lsk_io_read(p.c_str(), 0, (int64_t)(w.size() * 4), w.data(), 3) == 0);
  CHECK(memcmp(v.data(), w.data(), v.size() * 4) == 0);
  unlink(p.c_str());
}

static void test_filelist() {
  const char text[] = "a.float3\r\n\nb.float3\nc.float3";  // CRLF, blank, no trailing \n
  std::string p = tmpfile_with(text, sizeof(text) - 1);
  char buf[256];
  int64_t n = lsk_io_read_filelist(p.c_str(), buf, sizeof(buf));
  CHECK(n == 3);
  CHECK(std::string(buf) == "a.float3\nb.float3\nc.float3");
  unlink(p.c_str());
}

static int parse(int variant, std::vector<const char *> av, lsk_cli_args *a, std::string *err) {
  char e[2048] = {0};
  int rc = lsk_cli_parse(variant, (int)av.size(), av.data(), a, e, sizeof(e));
  *err = e;
  return rc;
}

static void test_cli() {
  lsk_cli_args a;
  std::string err;
  CHECK(parse(0, {"x", "-k", "5", "in1", "-o", "out", "in2", "-r", "0.5", "-g", "8"}, &a, &err) == 0);
  CHECK(std::string(a.input) == "in2");  // last positional wins
  CHECK(std::string(a.output) == "out" && a.k == 5 && a.max_radius == 0.5f && a.gpu_affinity == 8);
  CHECK(parse(0, {"x", "-k", "5", "in"}, &a, &err) == 1);  // no -o
  CHECK(err.find("Error: ") == 0);
  CHECK(err.find("./mpiHugeQuery -k <k> [-r <maxRadius>] in.float3s -o out.dat") != std::string::npos);
  CHECK(parse(0, {"x", "-k", "0", "in", "-o", "o"}, &a, &err) == 1);  // k >= 1
  CHECK(parse(0, {"x", "--bogus", "in", "-o", "o", "-k", "1"}, &a, &err) == 1);
  CHECK(err.find("unknown cmdline arg") != std::string::npos);
  CHECK(parse(1, {"x", "-k", "1", "files.txt", "-o", "prefix"}, &a, &err) == 0);
  CHECK(parse(0, {"x", "in", "-o", "o", "-k", "3", "--mode", "ring", "--stats", "s.json"}, &a, &err) == 0);
  CHECK(std::string(a.mode) == "ring" && std::string(a.stats) == "s.json");
  CHECK(isinf(a.max_radius));
}

// reference computePermutation written out independently (glibc rand())
static std::vector<int> ref_perm(int rank, int size) {
  srand(rank + 0x1234567);
  for (int i = 0; i < 10; i++) rand();
  std::vector<int> r(size);
  for (int i = 0; i < size; i++) r[i] = i;
  for (int i = size - 1; i > 0; --i) std::swap(r[rand() % i], r[i]);
  return r;
}

static void test_peer_schedule() {
  for (int size : {1, 2, 3, 8, 12, 64}) {
    for (int rank = 0; rank < size; rank++) {
      std::vector<int> got(size);
      lsk_peer_permutation(rank, size, got.data());
      CHECK(got == ref_perm(rank, size));
      // Sattolo: one single cycle through all ranks
      if (size > 1) {
        int steps = 0, at = 0;
        do {
          at = got[at];
          steps++;
        } while (at != 0 && steps <= size);
        CHECK(steps == size);
      }
    }
  }
  const float a[6] = {0, 0, 0, 1, 1, 1}, b[6] = {2, 0, 0, 3, 1, 1}, c[6] = {4, 3, 0, 5, 4, 1};
  CHECK(lsk_box_distance(a, b) == 1.f);
  CHECK(fabsf(lsk_box_distance(a, c) - sqrtf(9.f + 4.f)) < 1e-6f);
  CHECK(lsk_box_distance(a, a) == 0.f);
  // choose: closest unseen within cutoff; ties -> first in permutation order
  float boxes[4 * 6] = {0, 0, 0, 1, 1, 1,  2, 0, 0, 3, 1, 1,  0, 2, 0, 1, 3, 1,  9, 9, 9, 10, 10, 10};
  uint8_t seen[4] = {1, 0, 0, 0};
  int perm[4] = {0, 2, 1, 3};
  CHECK(lsk_peer_choose(boxes, boxes, 4, 5.f, seen, perm) == 2);  // 1 and 2 tie at 1.0
  seen[2] = 1;
  CHECK(lsk_peer_choose(boxes, boxes, 4, 5.f, seen, perm) == 1);
  seen[1] = 1;
  CHECK(lsk_peer_choose(boxes, boxes, 4, 5.f, seen, perm) == -1);  // 3 is beyond the cutoff
  CHECK(lsk_peer_choose(boxes, boxes, 4, 100.f, seen, perm) == 3);
}

static void test_oracles_agree() {
  std::mt19937 rng(5);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  const int n = 3000;
  std::vector<float> p(3 * n);
  for (auto &x : p) x = U(rng);
  for (int i = 0; i < 50; i++) {  // exact duplicates
    p[3 * (n - 1 - i)] = p[3 * i];
    p[3 * (n - 1 - i) + 1] = p[3 * i + 1];
    p[3 * (n - 1 - i) + 2] = p[3 * i + 2];
  }
  std::vector<float> o1(n), o2(n);
  for (int k : {1, 7, 100}) {
    for (float r : {INFINITY, 0.03f}) {
      const float cut2 = isinf(r) ? INFINITY : r * r;
      lsk_cpu_kth_brute(p.data(), n, p.data(), n, k, cut2, o1.data(), 4);
      lsk_cpu_kth_kdtree(p.data(), n, p.data(), n, k, cut2, o2.data(), 4);
      CHECK(memcmp(o1.data(), o2.data(), n * 4) == 0);
      for (int i = 0; i < n; i++) CHECK(o1[i] <= cut2);
    }
  }
  lsk_cpu_kth_brute(p.data(), 10, p.data(), 10, 11, INFINITY, o1.data(), 1);  // k > n -> inf
  for (int i = 0; i < 10; i++) CHECK(isinf(o1[i]));
}

int main() {
  test_partition();
  test_read_write_roundtrip();
  test_filelist();
  test_cli();
  test_peer_schedule();
  test_oracles_agree();
  if (g_fail) {
    fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  printf("host tests passed\n");
  return 0;
}
