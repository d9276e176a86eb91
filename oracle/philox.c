/* ORACLE -- test infrastructure only.
 * Plain-C restatement of numpy's Philox4x64-10 bit generator and
 * Generator.random() as used by cubed/random.py:31-36
 * (Generator(Philox(key=root_seed + block_offset)).random(shape)):
 *   key = [low 64 bits, high 64 bits] of the 128-bit integer;
 *   counter starts at 0 and is incremented BEFORE each 4-word block;
 *   random() = (next_uint64 >> 11) * 2^-53.
 * Pinned against numpy by tests/golden/philox_blocks.json
 * (tests/test_oracle.py).  Built by oracle/Makefile into oracle/_ref/. */
#include <stdint.h>

static void mulhilo(uint64_t a, uint64_t b, uint64_t* hi, uint64_t* lo) {
  __uint128_t p = (__uint128_t)a * b;
  *hi = (uint64_t)(p >> 64);
  *lo = (uint64_t)p;
}

static void philox4x64_10(const uint64_t ctr_in[4], uint64_t k0, uint64_t k1, uint64_t out[4]) {
  uint64_t x0 = ctr_in[0], x1 = ctr_in[1], x2 = ctr_in[2], x3 = ctr_in[3];
  for (int r = 0; r < 10; ++r) {
    uint64_t hi0, lo0, hi1, lo1;
    mulhilo(0xD2E7470EE14C6C93ull, x0, &hi0, &lo0);
    mulhilo(0xCA5A826395121157ull, x2, &hi1, &lo1);
    uint64_t y0 = hi1 ^ x1 ^ k0, y2 = hi0 ^ x3 ^ k1;
    x0 = y0; x1 = lo1; x2 = y2; x3 = lo0;
    k0 += 0x9E3779B97F4A7C15ull;
    k1 += 0xBB67AE8584CAA73Bull;
  }
  out[0] = x0; out[1] = x1; out[2] = x2; out[3] = x3;
}

/* Fill out[0..n) with the stream of key (k0, k1), starting at element start. */
void oracle_philox_uniform(uint64_t k0, uint64_t k1, int64_t start, int64_t n, double* out) {
  uint64_t ctr[4] = {0, 0, 0, 0};
  uint64_t buf[4];
  for (int64_t i = 0; i < n; ++i) {
    int64_t e = start + i;
    uint64_t blk = (uint64_t)(e / 4) + 1;
    ctr[0] = blk; ctr[1] = (blk == 0); ctr[2] = 0; ctr[3] = 0;
    philox4x64_10(ctr, k0, k1, buf);
    out[i] = (double)(buf[e % 4] >> 11) * (1.0 / 9007199254740992.0);
  }
}
