// Sanitizer fuzz driver for plato_ingest_parse / plato_ingest_gather (host code).
// Built by tests/test_ingest_sanitize.py with -fsanitize=address,undefined
// together with plato_amd/csrc/ingest.cpp.  For every sample file: parse all
// prefixes and thousands of random byte mutations; gather whatever parses;
// read the file back through plato_ingest_read_fd (short and exact lengths)
// and re-join it from random chunkings with plato_ingest_join.
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "plato_ingest.h"

static void exercise(const std::vector<uint8_t>& b, size_t* ok, size_t* err) {
  std::vector<plato_ingest_tensor> t(256);
  const int n = plato_ingest_parse(b.data(), b.size(), t.data(), int(t.size()));
  if (n < 0) {
    ++*err;
    return;
  }
  ++*ok;
  std::vector<uint64_t> off(static_cast<size_t>(n));
  uint64_t total = 0;
  for (int i = 0; i < n; ++i) {
    off[size_t(i)] = total;
    total += t[size_t(i)].numel * uint64_t(t[size_t(i)].element_size);
  }
  if (total > (uint64_t(1) << 28)) return;
  std::vector<uint8_t> dst(size_t(total) + 1);
  plato_ingest_gather(b.data(), b.size(), t.data(), n, off.data(), dst.data(), dst.size(), 4);
}

int main(int argc, char** argv) {
  size_t ok = 0, err = 0;
  std::mt19937_64 rng(1234);
  for (int a = 1; a < argc; ++a) {
    FILE* f = std::fopen(argv[a], "rb");
    if (!f) return 2;
    std::vector<uint8_t> data;
    uint8_t buf[65536];
    size_t got;
    while ((got = std::fread(buf, 1, sizeof(buf), f)) > 0) data.insert(data.end(), buf, buf + got);
    std::fclose(f);
    for (size_t cut = 0; cut <= data.size(); cut += (data.size() > 4096 ? 7 : 1)) {
      std::vector<uint8_t> p(data.begin(), data.begin() + long(cut));
      exercise(p, &ok, &err);
    }
    // read_fd: whole file on 1 and 4 threads, then one byte past the end (must fail)
    const int fd = ::open(argv[a], O_RDONLY);
    if (fd < 0) return 3;
    for (int threads : {1, 4}) {
      std::vector<uint8_t> back(data.size() + 1);
      if (plato_ingest_read_fd(fd, back.data(), data.size(), threads) != int64_t(data.size())) return 4;
      if (std::memcmp(back.data(), data.data(), data.size()) != 0) return 5;
      if (plato_ingest_read_fd(fd, back.data(), data.size() + 1, threads) != PLATO_INGEST_EIO) return 6;
    }
    ::close(fd);
    // join: random chunkings of the file reassemble it byte for byte
    for (int rep = 0; rep < 50; ++rep) {
      std::vector<const uint8_t*> ptrs;
      std::vector<size_t> lens;
      for (size_t pos = 0; pos < data.size();) {
        const size_t len = std::min(data.size() - pos, size_t(1 + rng() % 5000));
        ptrs.push_back(data.data() + pos);
        lens.push_back(len);
        pos += len;
      }
      std::vector<uint8_t> joined(data.size());
      if (plato_ingest_join(ptrs.data(), lens.data(), int(ptrs.size()), joined.data(), joined.size(), 4) != 0) return 7;
      if (joined != data) return 8;
      if (!ptrs.empty() &&
          plato_ingest_join(ptrs.data(), lens.data(), int(ptrs.size()), joined.data(), joined.size() - 1, 4) !=
              PLATO_INGEST_ECAPACITY)
        return 9;
    }
    for (int m = 0; m < 4000; ++m) {
      std::vector<uint8_t> p = data;
      const int flips = 1 + int(rng() % 4);
      for (int k = 0; k < flips; ++k) p[rng() % p.size()] = uint8_t(rng());
      exercise(p, &ok, &err);
    }
  }
  std::printf("FUZZ_OK %zu %zu\n", ok, err);
  return 0;
}
