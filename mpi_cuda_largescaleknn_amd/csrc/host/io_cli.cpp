// Host I/O, CLI grammar and the prePartitioned peer schedule.
//
// Reference parity (behaviour, not code):
//   - CLI loop: unorderedDataVariant.cu:114-135 / prePartitionedDataVariant.cu:185-206
//   - usage():  unorderedDataVariant.cu:66-71 (stderr text, exit(error.empty()?0:1))
//   - readFilePortion: unorderedDataVariant.cu:42-63 (size_t partition math)
//   - readListOfFileNames: prePartitionedDataVariant.cu:114-126 (we also accept an
//     unterminated last line and strip CR — SURVEY D11)
//   - computePermutation / computeDistance / computeMyPeer:
//     prePartitionedDataVariant.cu:136-174
#include "lsk_host.h"
#include "../common.h"

#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <string>
#include <thread>
#include <vector>

extern "C" int lsk_host_abi_version(void) { return 2; }

// ============================================================================ CLI
namespace {

const char *kSynopsis = "./mpiHugeQuery -k <k> [-r <maxRadius>] in.float3s -o out.dat";

int usage_error(const std::string &msg, char *err, int errlen) {
  std::string text = "Error: " + msg + "\n\n" + kSynopsis + "\n";
  if (err && errlen > 0) {
    std::snprintf(err, (size_t)errlen, "%s", text.c_str());
  }
  return msg.empty() ? 0 : 1;
}

void copy_str(char *dst, size_t cap, const std::string &s) {
  std::snprintf(dst, cap, "%s", s.c_str());
}

}  // namespace

extern "C" int lsk_cli_parse(int variant, int argc, const char **argv, lsk_cli_args *out,
                             char *err, int errlen) {
  std::memset(out, 0, sizeof(*out));
  out->max_radius = std::numeric_limits<float>::infinity();
  copy_str(out->mode, sizeof(out->mode), "auto");
  copy_str(out->device, sizeof(out->device), "auto");
  copy_str(out->bootstrap, sizeof(out->bootstrap), "auto");
  copy_str(out->balance, sizeof(out->balance), "auto");
  std::string input, output;

  auto need_value = [&](int i, const std::string &flag) -> bool {
    if (i + 1 >= argc) {
      usage_error("missing value for '" + flag + "'", err, errlen);
      return false;
    }
    return true;
  };

  for (int i = 1; i < argc; i++) {
    const std::string arg = argv[i] ? argv[i] : "";
    if (arg == "-o") {
      if (!need_value(i, arg)) return 1;
      output = argv[++i];
    } else if (arg.empty() || arg[0] != '-') {
      input = arg;  // last positional wins (reference behaviour)
    } else if (arg == "-r") {
      if (!need_value(i, arg)) return 1;
      out->max_radius = (float)std::atof(argv[++i]);
    } else if (arg == "-g") {
      if (!need_value(i, arg)) return 1;
      out->gpu_affinity = std::atoi(argv[++i]);
    } else if (arg == "-k") {
      if (!need_value(i, arg)) return 1;
      out->k = std::atoi(argv[++i]);
    } else if (arg == "--mode") {
      if (!need_value(i, arg)) return 1;
      std::string m = argv[++i];
      if (m != "auto" && m != "halo" && m != "ring" && m != "peer")
        return usage_error("invalid --mode '" + m + "' (auto|halo|ring|peer)", err, errlen);
      copy_str(out->mode, sizeof(out->mode), m);
    } else if (arg == "--device") {
      if (!need_value(i, arg)) return 1;
      std::string d = argv[++i];
      if (d != "auto" && d != "cuda" && d != "cpu")
        return usage_error("invalid --device '" + d + "' (auto|cuda|cpu)", err, errlen);
      copy_str(out->device, sizeof(out->device), d);
    } else if (arg == "--stats") {
      if (!need_value(i, arg)) return 1;
      copy_str(out->stats, sizeof(out->stats), argv[++i]);
    } else if (arg == "--bootstrap") {
      if (!need_value(i, arg)) return 1;
      std::string b = argv[++i];
      if (b != "auto" && b != "env" && b != "mpi" && b != "spawn")
        return usage_error("invalid --bootstrap '" + b + "' (auto|env|mpi|spawn)", err, errlen);
      copy_str(out->bootstrap, sizeof(out->bootstrap), b);
    } else if (arg == "--nproc") {
      if (!need_value(i, arg)) return 1;
      out->nproc = std::atoi(argv[++i]);
      if (out->nproc < 1 || out->nproc > 1024)
        return usage_error("invalid --nproc (1..1024)", err, errlen);
    } else if (arg == "--device-map") {
      if (!need_value(i, arg)) return 1;
      std::string m = argv[++i];
      bool ok = !m.empty() && m.size() < sizeof(out->device_map) && m.front() != ',' && m.back() != ',';
      for (size_t c = 0; ok && c < m.size(); c++)
        ok = (m[c] >= '0' && m[c] <= '9') || (m[c] == ',' && m[c - 1] != ',');
      if (!ok) return usage_error("invalid --device-map '" + m + "' (e.g. 0,1,2,3)", err, errlen);
      copy_str(out->device_map, sizeof(out->device_map), m);
    } else if (arg == "--balance") {
      if (!need_value(i, arg)) return 1;
      std::string b = argv[++i];
      if (b != "auto" && b != "on" && b != "off")
        return usage_error("invalid --balance '" + b + "' (auto|on|off)", err, errlen);
      copy_str(out->balance, sizeof(out->balance), b);
    } else if (arg == "-v" || arg == "--verbose") {
      out->verbose = 1;
    } else {
      return usage_error("unknown cmdline arg '" + arg + "'", err, errlen);
    }
  }
  if (input.empty())
    return usage_error(variant == 0 ? "no input file name specified"
                                    : "no input file name specified (should be a text file "
                                      "with list of input files)",
                       err, errlen);
  if (output.empty())
    return usage_error(variant == 0 ? "no output file name specified"
                                    : "no output file(s) prefix specified",
                       err, errlen);
  if (out->k < 1) return usage_error("no k specified, or invalid k value", err, errlen);
  if ((std::string(out->bootstrap) == "spawn") != (out->nproc > 0))
    return usage_error("--bootstrap spawn and --nproc N go together", err, errlen);
  if (input.size() >= sizeof(out->input) || output.size() >= sizeof(out->output))
    return usage_error("path too long", err, errlen);
  copy_str(out->input, sizeof(out->input), input);
  copy_str(out->output, sizeof(out->output), output);
  return 0;
}

// ============================================================================ I/O
namespace {

int64_t file_size(const char *path) {
  struct stat st;
  if (stat(path, &st) != 0) return -errno;
  return (int64_t)st.st_size;
}

// Splits [0, nbytes) over nthreads, each issuing pread/pwrite loops on its own range.
template <typename F>
int parallel_chunks(int64_t nbytes, int nthreads, F &&fn) {
  if (nthreads < 1) nthreads = 1;
  const int64_t min_chunk = 8ll << 20;
  int64_t nt = std::min<int64_t>(nthreads, std::max<int64_t>(1, nbytes / min_chunk));
  std::atomic<int> rc{0};
  std::vector<std::thread> th;
  for (int64_t t = 0; t < nt; t++) {
    int64_t b = nbytes * t / nt, e = nbytes * (t + 1) / nt;
    th.emplace_back([&, b, e] {
      int r = fn(b, e);
      if (r) rc.store(r);
    });
  }
  for (auto &x : th) x.join();
  return rc.load();
}

}  // namespace

extern "C" int lsk_io_portion(const char *path, int64_t rank, int64_t size, int64_t recsize,
                              int64_t *begin, int64_t *count, int64_t *total) {
  int64_t bytes = file_size(path);
  if (bytes < 0) return (int)bytes;
  if (size < 1 || rank < 0 || rank >= size || recsize < 1) return -EINVAL;
  const uint64_t num = (uint64_t)bytes / (uint64_t)recsize;  // trailing partial record ignored
  // floor(num*r/P) in 128-bit to stay exact for any file size.
  const uint64_t b = (uint64_t)(((__uint128_t)num * (uint64_t)rank) / (uint64_t)size);
  const uint64_t e = (uint64_t)(((__uint128_t)num * (uint64_t)(rank + 1)) / (uint64_t)size);
  if (begin) *begin = (int64_t)b;
  if (count) *count = (int64_t)(e - b);
  if (total) *total = (int64_t)num;
  return 0;
}

extern "C" int lsk_io_read(const char *path, int64_t offset, int64_t nbytes, void *dst,
                           int nthreads) {
  if (nbytes <= 0) return 0;
  int fd = open(path, O_RDONLY);
  if (fd < 0) return -errno;
  int rc = parallel_chunks(nbytes, nthreads, [&](int64_t b, int64_t e) -> int {
    char *p = (char *)dst;
    while (b < e) {
      ssize_t r = pread(fd, p + b, (size_t)std::min<int64_t>(e - b, 1ll << 30), offset + b);
      if (r < 0) {
        if (errno == EINTR) continue;
        return -errno;
      }
      if (r == 0) return -EIO;  // file shorter than expected
      b += r;
    }
    return 0;
  });
  close(fd);
  return rc;
}

extern "C" int lsk_io_write(const char *path, int64_t offset, const void *src, int64_t nbytes,
                            int flags, int64_t total_size, int nthreads) {
  int oflags = O_WRONLY | O_CREAT;
  if (flags & 1) oflags |= O_TRUNC;
  int fd = open(path, oflags, 0644);
  if (fd < 0) return -errno;
  if ((flags & 2) && total_size >= 0) {
    if (ftruncate(fd, total_size) != 0) {
      int e = -errno;
      close(fd);
      return e;
    }
  }
  int rc = 0;
  if (nbytes > 0) {
    rc = parallel_chunks(nbytes, nthreads, [&](int64_t b, int64_t e) -> int {
      const char *p = (const char *)src;
      while (b < e) {
        ssize_t r =
            pwrite(fd, p + b, (size_t)std::min<int64_t>(e - b, 1ll << 30), offset + b);
        if (r < 0) {
          if (errno == EINTR) continue;
          return -errno;
        }
        b += r;
      }
      return 0;
    });
  }
  if (close(fd) != 0 && rc == 0) rc = -errno;
  return rc;
}

extern "C" int64_t lsk_io_read_filelist(const char *path, char *buf, int64_t buflen) {
  std::ifstream in(path);
  if (!in) return -ENOENT;
  std::vector<std::string> names;
  std::string line;
  while (std::getline(in, line)) {
    while (!line.empty() && (line.back() == '\r' || line.back() == '\n')) line.pop_back();
    if (line.empty()) continue;  // blank lines carry no rank
    names.push_back(line);
  }
  std::string joined;
  for (size_t i = 0; i < names.size(); i++) {
    if (i) joined += '\n';
    joined += names[i];
  }
  if ((int64_t)joined.size() + 1 > buflen) return -((int64_t)joined.size() + 1) - 1000000;
  std::memcpy(buf, joined.c_str(), joined.size() + 1);
  return (int64_t)names.size();
}

// ============================================================================ peer schedule
extern "C" void lsk_peer_permutation(int rank, int size, int *out) {
  // glibc rand() sequence, exactly as the reference seeds it.
  std::srand((unsigned)(rank + 0x1234567));
  for (int i = 0; i < 10; i++) (void)std::rand();
  for (int i = 0; i < size; i++) out[i] = i;
  for (int i = size - 1; i > 0; --i) {
    int other = std::rand() % i;  // Sattolo: % i, single-cycle permutation
    std::swap(out[other], out[i]);
  }
}

extern "C" float lsk_box_distance(const float *a, const float *b) {
  lsk::box3f A{{a[0], a[1], a[2]}, {a[3], a[4], a[5]}};
  lsk::box3f B{{b[0], b[1], b[2]}, {b[3], b[4], b[5]}};
  // The reference evaluates sqrtf(dx*dx+dy*dy+dz*dz); the value only steers the
  // schedule (never the kNN result), so the canonical dist2 is used here.
  return sqrtf(lsk::box_box_dist2(A, B));
}

extern "C" int lsk_peer_choose(const float *my_box, const float *all_boxes, int size,
                               float cutoff, const uint8_t *seen, const int *perm) {
  int best = -1;
  float closest = std::numeric_limits<float>::infinity();
  for (int i = 0; i < size; i++) {
    int peer = perm[i];
    if (seen[peer]) continue;
    float d = lsk_box_distance(my_box, all_boxes + 6 * peer);
    if (d >= cutoff) continue;
    if (d >= closest) continue;
    closest = d;
    best = peer;
  }
  return best;
}
