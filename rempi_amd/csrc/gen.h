// gen.h -- the synthetic per-rank MPI event traces of the benchmark workload, defined as closed-form
// functions of (rank, index) so that the host (tests, CPU baseline) and the device (bench)
// produce bit-identical streams.  Definition, in words:
//
//  * A rank r of a job of W ranks has S' = min(S, W-1) senders; sender j sends from rank
//    (r + 1 + j) mod W and belongs to matching set t = j mod T' (T' = min(T, S')).
//  * Set t's messages m = 0,1,.. come in blocks of n_t = #senders of t: message m is from
//    sender j = t + T'*(m mod n_t) with Lamport clock 15 + 5b + h(j,b) mod 5, b = m / n_t
//    (strictly increasing per sender, +1..+9 per message).
//  * Arrival key = clock + h(t,m) mod (J+1); a set's matched receives are observed in
//    (arrival key, m) order.
//  * The stream is a sequence of matching-function calls ("frames").  Frame f serves set
//    h(f) mod T'; with probability 1/5 it first records an unmatched poll of that set
//    (event_count 1 + min(geometric(1/2), 62)); it then records g matched receives of
//    the set (g = 1, or 2..4 with probability 1/10: a Testsome with with_next = 1 on all
//    but the last), index = h(f,i) mod 16.  Frames are added while the record count stays
//    <= events_per_rank.
//  * Records are canonical: no two consecutive records are equal in fields 1..7.
#pragma once
#include <stdint.h>

#include "hash_order.h"  // CDCX_HD

namespace cdcx {
namespace gen {

enum : uint64_t { kTagSet = 1, kTagUnm = 2, kTagGrp = 3, kTagGsz = 4, kTagCnt = 5, kTagClk = 6, kTagJit = 7, kTagIdx = 8 };

CDCX_HD inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
CDCX_HD inline uint64_t rank_seed(int32_t r, uint64_t salt) {
  return 0x5EEDC0DEull ^ ((uint64_t)(uint32_t)r * 0x9E3779B97F4A7C15ull) ^ salt;
}
CDCX_HD inline uint64_t h(uint64_t seed, uint64_t tag, uint64_t a, uint64_t b) {
  return mix64(mix64(seed ^ (tag * 0xD1B54A32D192ED03ull)) ^ (a * 0xA24BAED4963EE407ull) ^ (b * 0x9FB21C651E98DF25ull));
}

struct Shape {
  int32_t W, S, T, J;
  CDCX_HD int32_t senders_of(int32_t t) const { return (S - t + T - 1) / T; }
};

CDCX_HD inline Shape shape(int32_t world, int32_t senders, int32_t sets, int32_t jitter) {
  Shape s;
  s.W = world;
  s.S = senders < world - 1 ? senders : world - 1;
  if (s.S < 1) s.S = 1;
  s.T = sets < s.S ? sets : s.S;
  if (s.T < 1) s.T = 1;
  s.J = jitter < 0 ? 0 : jitter;
  return s;
}

struct Frame {
  int32_t set;
  int32_t unmatched;  // 0/1
  int32_t g;          // matched receives
  int32_t count;      // event_count of the poll
};

CDCX_HD inline Frame frame(uint64_t seed, const Shape& sh, int64_t f) {
  Frame fr;
  fr.set = (int32_t)(h(seed, kTagSet, f, 0) % (uint64_t)sh.T);
  fr.unmatched = (h(seed, kTagUnm, f, 0) % 5) == 0;
  fr.g = (h(seed, kTagGrp, f, 0) % 10 == 0) ? 2 + (int32_t)(h(seed, kTagGsz, f, 0) % 3) : 1;
  const uint64_t c = h(seed, kTagCnt, f, 0) | (1ull << 62);
  int32_t tz = 0;
  while (!((c >> tz) & 1)) tz++;
  fr.count = 1 + tz;
  return fr;
}

struct Msg {
  int32_t src;
  int32_t clock;
  int64_t akey;
};

CDCX_HD inline Msg message(uint64_t seed, const Shape& sh, int32_t r, int32_t t, int64_t m) {
  const int32_t nt = sh.senders_of(t);
  const int64_t b = m / nt;
  const int32_t j = t + sh.T * (int32_t)(m % nt);
  Msg g;
  g.src = (int32_t)(((int64_t)r + 1 + j) % sh.W);
  g.clock = (int32_t)(15 + 5 * b + (int64_t)(h(seed, kTagClk, (uint64_t)j, (uint64_t)b) % 5));
  g.akey = (int64_t)g.clock + (int64_t)(h(seed, kTagJit, (uint64_t)t, (uint64_t)m) % (uint64_t)(sh.J + 1));
  return g;
}

// Blocks on either side of a message's block that can hold messages arriving before /
// after it; everything further left arrives earlier, further right later.
CDCX_HD inline int64_t window_blocks(const Shape& sh) { return (4 + sh.J) / 5 + 2; }

CDCX_HD inline int32_t index_of(uint64_t seed, int64_t f, int32_t i) {
  return (int32_t)(h(seed, kTagIdx, (uint64_t)f, (uint64_t)i) % 16);
}

}  // namespace gen
}  // namespace cdcx
