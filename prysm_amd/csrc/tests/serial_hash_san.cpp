// Host-only sanitizer driver for the serial hasher (serial_hash.cpp): ASan/UBSan and TSan
// builds (Makefile targets san-asan / san-tsan) hash messages of every block-boundary length
// single-threaded and through the multi-threaded SerialHashJob, and check both against each
// other and against RFC 7693's BLAKE2b-512("abc").  Exit status 0 = clean and consistent.
#include <cstdio>
#include <cstring>
#include <vector>

#include "../serial_hash.h"

int main() {
  static const uint8_t kAbc[64] = {
      0xba, 0x80, 0xa5, 0x3f, 0x98, 0x1c, 0x4d, 0x0d, 0x6a, 0x27, 0x97, 0xb6, 0x9f, 0x12, 0xf6, 0xe9,
      0x4c, 0x21, 0x2f, 0x14, 0x68, 0x5a, 0xc4, 0xb7, 0x4b, 0x12, 0xbb, 0x6f, 0xdb, 0xff, 0xa2, 0xd1,
      0x7d, 0x87, 0xc5, 0x39, 0x2a, 0xab, 0x79, 0x2d, 0xc2, 0x52, 0xd5, 0xde, 0x45, 0x33, 0xcc, 0x95,
      0x18, 0xd3, 0x8a, 0xa8, 0xdb, 0xf1, 0x92, 0x5a, 0xb9, 0x23, 0x86, 0xed, 0xd4, 0x00, 0x99, 0x23};
  uint8_t d[64];
  pz::host_blake2b512(reinterpret_cast<const uint8_t*>("abc"), 3, d);
  if (std::memcmp(d, kAbc, 64)) {
    std::puts("FAIL abc");
    return 1;
  }
  std::vector<uint8_t> data;
  std::vector<uint64_t> offs{0}, which;
  for (int len = 0; len <= 1100; ++len) {  // every block boundary several times
    for (int i = 0; i < len; ++i) data.push_back((uint8_t)(len * 31 + i * 7));
    offs.push_back(data.size());
    which.push_back(offs.size() - 2);
  }
  const size_t n = offs.size() - 1;
  std::vector<uint8_t> one(n * 64), many(n * 64);
  for (size_t i = 0; i < n; ++i) pz::host_blake2b512(data.data() + offs[i], offs[i + 1] - offs[i], &one[i * 64]);
  {
    pz::SerialHashJob job;
    job.start(data.data(), offs.data(), which, many.data(), 64);
  }  // joined
  if (one != many) {
    std::puts("FAIL threaded");
    return 1;
  }
  std::printf("ok %zu messages\n", n);
  return 0;
}
