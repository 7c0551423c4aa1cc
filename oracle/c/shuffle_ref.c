/* ORACLE (test infrastructure only) — C restatement of utils.ShuffleIndices
 * (beacon-chain/utils/shuffle.go:14-33), verbatim in its arithmetic: the seed stream is
 * blake2b.Sum512(seed) (:19), each of the 21 swap numbers is the byte-wrapped sum of three
 * seed bytes (:25-26, j = 0, 3, .., 60), and position i swaps with sw % (n - i) + i (:28-31),
 * i = 0 .. n-2.  Used as the checker of pz_shuffle_indices at any n and as its CPU baseline. */
#include <stdint.h>
#include <stddef.h>

void oracle_blake2b512(const uint8_t* msg, uint64_t len, uint8_t out[64]);

int oracle_shuffle_indices(const uint8_t seed[32], uint32_t* list, uint64_t n) {
  if (n > 4194304ull) return -3; /* params.MaxValidators (utils/shuffle.go:15-17) */
  uint8_t hs[64];
  oracle_blake2b512(seed, 32, hs);
  for (uint64_t i = 0; i + 1 < n; ++i) {
    for (int j = 0; j + 3 < 64; j += 3) {
      const uint8_t sw = (uint8_t)(hs[j] + hs[j + 1] + hs[j + 2]);
      const uint64_t rem = n - i;
      const uint64_t p = (uint64_t)sw % rem + i;
      const uint32_t t = list[i];
      list[i] = list[p];
      list[p] = t;
    }
  }
  return 0;
}
