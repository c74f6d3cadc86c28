// decode_lanes.hip -- the permutation rebuild's pair segments (decode.hip) with one segment per
// LANE: 64 segments per wave, the list of cdc_prepare_decode_indices
// (rempi_encoder_cdc.cpp:1301-1386) as a doubly linked list in LDS.
//
// The 16-lane groups of k_dec_perm_seg spend about twenty vector instructions per pair, most of
// them on control that four groups share.  Here one vector instruction advances 64 segments,
// and a move is what it is in the reference: unlink the element, follow `delay` links, link it
// in again.  Per lane the list lives in a ring of 128 two-byte nodes {next, previous}, node of
// element e at slot e & 127; the element of a slot follows from the slot and `hi`, the next
// element not yet in the list: the live elements all lie in [hi - 128, hi).  Elements from `hi`
// on are untouched and follow the list's tail in order; they are linked in ("loaded") as pairs
// come near them, kLAhead ahead of the pair's id and on demand when a walk runs off the tail.
// The head of the list is the first position that is not final yet (`spos`): when a slot is
// needed for a new element, heads are settled -- written to cinv, their slot freed -- until
// that slot is free.  Node of (slot s, lane l) is the half word s * 64 + l of the LDS image: a
// lane's accesses stay in its own bank pair whatever the slot.
//
// Segments, replay, ownership of list positions and the state check are those of decode.hip:
// the segment replays the kSegWarm pairs before its own from the untouched list without
// writing (a pair that does not fit is skipped and the list left as it was), settles up to its
// first owned position `own` and writes the kSegWin positions from there to dumpW; it never
// settles past `cap`, the next segment's first position, and writes the positions from there to
// dumpT when it is done.  k_dec_perm_check compares, k_dec_perm_seg<2> reruns what differs.
// A pair that reaches before the head (the positions there are final), a walk past the last
// element of the list, an id that is not in the list or a ring that cannot take the next
// element without settling past `cap` fail the segment's unit for this tier.
// Only cinv (position -> element) is written here; k_dec_perm_inv turns it into perm.
#include <hip/hip_runtime.h>

#include "cdcx_device.h"
#include "cdcx_kernels.h"

namespace cdcx {

namespace {
constexpr int32_t kLSlots = 128;    // ring slots per lane
constexpr int32_t kLAhead = 40;     // elements linked in ahead of a pair's id
constexpr int32_t kLNone = 0x80;    // no neighbour: before the head / after the tail
constexpr uint32_t kLDead = 0xFFFF;  // the slot holds no live element
constexpr int32_t kLStage = 8;      // pairs per lane fetched at a time
constexpr int32_t kLGap = 512;      // an id this far past `hi` is reached by a jump, not link by link
}  // namespace

__global__ void __launch_bounds__(64) k_dec_perm_lanes(DUnit* __restrict__ units, const DSeg* __restrict__ segs,
                                                       int64_t nsegs, const uint8_t* __restrict__ in,
                                                       const int64_t* __restrict__ pcar, int32_t* __restrict__ cinv,
                                                       int32_t* __restrict__ dumpT, int32_t* __restrict__ dumpW,
                                                       int32_t* __restrict__ nfail) {
  __shared__ uint16_t node_s[kLSlots * 64];
  __shared__ int32_t stage_s[2 * kLStage * 64];
  uint8_t* const nb = reinterpret_cast<uint8_t*>(node_s);
  const int l = threadIdx.x;
  const int64_t gi = (int64_t)blockIdx.x * 64 + l;
  DSeg sd{-1, 0, 0, 0, 0, kSegNoCap, 0, 0};
  int32_t M = 0, Pu = 0;
  int64_t key_off = 0, pair_off = 0;
  bool sim = false;
  if (gi < nsegs) {
    sd = segs[gi];
    const DUnit& u = units[sd.unit];
    sim = (u.fb == 0);
    M = u.M;
    Pu = u.P;
    key_off = u.key_off;
    pair_off = u.pair_off;
  }
  const bool wact = sim && sd.s > 0;            // replays kSegWarm pairs first
  const bool hasn = sd.cap != kSegNoCap;        // a segment follows: leave it the final state
  const int32_t ka = sd.ka, ke = sim ? sd.ke : sd.ka;
  const int32_t klo = wact ? ka - kSegWarm : ka;
  const int32_t own = sd.own, cap = sd.cap;
  const int32_t lim_main = min(M, cap);         // positions below it are this segment's to settle
  // inverse LP state, low words (the moves use the low 32 bits; rempi_compression_util.cpp:157-168)
  uint32_t zi = 0, xi = 0, zd = 0, xd = 0;
  if (wact) {
    const int64_t* o = pcar + 4 * gi;
    zi = (uint32_t)o[0];
    xi = (uint32_t)o[1];
    zd = (uint32_t)o[2];
    xd = (uint32_t)o[3];
  }
  // every slot dead (the wave clears the whole image, 16 bytes per lane and step)
  for (int q = l; q < kLSlots * 64 * 2 / 16; q += 64) reinterpret_cast<int4*>(node_s)[q] = make_int4(-1, -1, -1, -1);
  int32_t head = kLNone, tail = kLNone;
  int32_t hi = wact ? sd.base0 : 0;  // next element to link in; spos + live elements == hi
  int32_t spos = hi;                 // list position of the head
  bool fail = !sim;

  auto node = [&](int32_t s) -> uint32_t { return node_s[s * 64 + l]; };
  auto set_node = [&](int32_t s, uint32_t v) { node_s[s * 64 + l] = (uint16_t)v; };
  auto set_next = [&](int32_t s, int32_t v) { nb[(s * 64 + l) * 2] = (uint8_t)v; };
  auto set_prev = [&](int32_t s, int32_t v) { nb[(s * 64 + l) * 2 + 1] = (uint8_t)v; };
  auto elem = [&](int32_t s) -> int32_t { return hi - kLSlots + ((s - hi) & (kLSlots - 1)); };

  // cinv[q] = q over [from, to) of the lanes in p: the wave writes each lane's stretch together
  auto fill = [&](bool p, int32_t from, int32_t to) {
    for (uint64_t m = __builtin_amdgcn_ballot_w64(p && from < to); m != 0; m &= m - 1) {
      const int src = __builtin_ctzll(m);
      const int32_t f = __builtin_amdgcn_readlane(from, src), t = __builtin_amdgcn_readlane(to, src);
      const int64_t ko = ((int64_t)__builtin_amdgcn_readlane((int32_t)(key_off >> 32), src) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int32_t)key_off, src);
      for (int32_t q = f + l; q < t; q += 64) cinv[ko + q] = q;
    }
  };
  // the head becomes final (lanes in p; they have a head)
  auto settle = [&](bool p, bool write) {
    const int32_t h = p ? head : 0;
    const uint32_t w = node(h);
    if (p) {
      if (write) cinv[key_off + spos] = elem(h);
      set_node(h, kLDead);
      const int32_t nx = (int32_t)(w & 0xFF);
      head = nx;
      if (nx != kLNone) set_prev(nx, kLNone);
      else tail = kLNone;
      spos++;
    }
  };
  // link in element hi (lanes in p; hi < M).  Its slot is freed first by settling heads, up to
  // position `lim`; where that does not free it the lane is returned in *stuck.
  // (lim <= spos: no settling -- a walk in flight holds links that settling could free)
  auto load = [&](bool p, int32_t lim, bool write, bool* stuck) {
    const int32_t s = hi & (kLSlots - 1);
    bool busy = p && node(s) != kLDead;
    while (__builtin_amdgcn_ballot_w64(busy)) {
      const bool can = busy && spos < lim && head != kLNone;
      *stuck |= busy && !can;
      settle(can, write);
      busy = can && node(s) != kLDead;
    }
    p = p && !*stuck;
    if (p) {
      set_node(s, ((uint32_t)tail << 8) | (uint32_t)kLNone);
      if (tail != kLNone) set_next(tail, s);
      else head = s;
      tail = s;
      hi++;
    }
  };
  // everything before position `upto` final: settle, and jump over untouched stretches
  auto settle_upto = [&](bool p, int32_t upto, bool write) {
    while (true) {
      const bool go = p && spos < upto;
      if (!__builtin_amdgcn_ballot_w64(go)) break;
      const bool empty = go && head == kLNone;  // (then spos == hi: the elements from here on are untouched)
      if (__builtin_amdgcn_ballot_w64(empty)) {
        if (write) fill(empty, hi, upto);
        if (empty) hi = spos = upto;
      }
      settle(go && !empty, write);
    }
  };
  // the kSegWin list positions from `from` (== spos) on, to dump[gi * kSegWin ...]
  auto dump_state = [&](bool p, int32_t* dump, int64_t g, int32_t from) {
    int32_t cur = head;
    for (int32_t q0 = 0; q0 < kSegWin; q0 += 4) {
      int32_t v[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const bool in_list = p && cur != kLNone;
        const uint32_t w = node(in_list ? cur : 0);
        v[q] = in_list ? elem(cur) : from + q0 + q;
        cur = in_list ? (int32_t)(w & 0xFF) : cur;
      }
      if (p) reinterpret_cast<int4*>(dump + g * kSegWin)[q0 / 4] = make_int4(v[0], v[1], v[2], v[3]);
    }
  };

  // the pairs' raw words: kLStage per lane and array at a time through LDS, fetched by the wave
  // with two lanes per segment so that every line is read once; the words of the next stretch
  // are in flight while this one is consumed
  int32_t ra[4], rb[4];  // raw id / delay words fetched ahead: pairs 4 * (l & 1) .. + 3 of segment (l >> 1) + 32 * half
  int32_t rc[4], rd[4];
  auto stage = [&]() {  // the fetched words into LDS: word of (pair q, segment s) at q * 64 + s
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int pq = 4 * (l & 1) + q;
      stage_s[pq * 64 + (l >> 1)] = ra[q];
      stage_s[(kLStage + pq) * 64 + (l >> 1)] = rb[q];
      stage_s[pq * 64 + (l >> 1) + 32] = rc[q];
      stage_s[(kLStage + pq) * 64 + (l >> 1) + 32] = rd[q];
    }
  };

  // one pair per lane.  WARM: the replay before the segment's own pairs (nothing is written, a
  // pair that does not fit is skipped with the list as it was, heads settle up to `own` only).
  auto round = [&](auto warm_c, bool inr, int32_t x, int32_t d) {
    constexpr bool WARM = decltype(warm_c)::value;
    const int32_t lim = WARM ? own : lim_main;
    bool act = inr && !fail;
    if (!WARM) {
      const bool badid = act && (uint32_t)x >= (uint32_t)M;
      fail |= badid;
      act = act && !badid;
    } else {
      act = act && (uint32_t)x < (uint32_t)M;
    }
    bool stuck = false;
    // an id far past the linked elements: everything before it is final, jump
    if (__builtin_amdgcn_ballot_w64(act && x - hi > kLGap)) {
      const bool far = act && x - hi > kLGap;
      const int32_t upto = min(x - kLAhead, lim);
      settle_upto(far, upto, !WARM);
      // (a jump that `lim` cut short leaves the links to be made one by one below, or the pair stuck)
    }
    // link in the elements up to kLAhead past the id
    const int32_t want = min(x + kLAhead, M - 1);
    while (true) {
      const bool need = act && !stuck && hi <= want;
      if (!__builtin_amdgcn_ballot_w64(need)) break;
      load(need, lim, !WARM, &stuck);
    }
    // take x out
    const int32_t s = x & (kLSlots - 1);
    const uint32_t wx = node(act ? s : 0);
    const bool gone = act && (stuck || x >= hi || wx == kLDead || x < hi - kLSlots);
    if (!WARM) fail |= gone;
    act = act && !gone;
    const int32_t a = (int32_t)(wx >> 8), b = (int32_t)(wx & 0xFF);
    if (act) {
      if (a == kLNone) head = b;
      else set_next(a, b);
      if (b == kLNone) tail = a;
      else set_prev(b, a);
    }
    // follow |d| links from its old successor
    int32_t cur = b, rem = d < 0 ? -d : d;
    const bool fwd = d > 0;
    bool lost = false;  // the walk left the list
    while (true) {
      const bool go = act && !lost && rem > 0;
      if (!__builtin_amdgcn_ballot_w64(go)) break;
      const bool off_end = go && fwd && cur == kLNone;  // past the tail: the next untouched element, if any
      if (__builtin_amdgcn_ballot_w64(off_end)) {
        const bool can = off_end && hi < M;
        lost |= off_end && !can;
        bool st = false;
        load(can, INT32_MIN, !WARM, &st);
        lost |= st;
        cur = (can && !st) ? tail : cur;
      }
      const bool stepf = go && fwd && !off_end;
      const bool stepb = go && !fwd;
      const uint32_t w = node((stepf || (stepb && cur != kLNone)) ? cur : 0);
      const int32_t nx = (int32_t)(w & 0xFF);
      const int32_t pv = (cur == kLNone) ? tail : (int32_t)(w >> 8);  // before "past the tail" comes the tail
      const bool before_head = stepb && pv == kLNone;
      lost |= before_head;
      cur = stepf ? nx : ((stepb && !before_head) ? pv : cur);
      rem -= (stepf || (stepb && !before_head)) ? 1 : 0;
    }
    if (!WARM) {
      fail |= act && lost;
      act = act && !lost;
    } else {
      cur = lost ? b : cur;  // skipped: back to where it was
    }
    // put x back in front of cur
    if (act) {
      const int32_t a2 = (cur == kLNone) ? tail : (int32_t)(node(cur) >> 8);
      set_node(s, ((uint32_t)a2 << 8) | (uint32_t)cur);
      if (a2 == kLNone) head = s;
      else set_next(a2, s);
      if (cur == kLNone) tail = s;
      else set_prev(cur, s);
    }
  };

  const std::integral_constant<bool, true> warm_t{};
  const std::integral_constant<bool, false> main_t{};
  auto next_pair = [&](int32_t r, int32_t* x, int32_t* d) {
    const int32_t yi = stage_s[(r & (kLStage - 1)) * 64 + l], yd = stage_s[(kLStage + (r & (kLStage - 1))) * 64 + l];
    zi += (uint32_t)yi;
    xi += zi;
    zd += (uint32_t)yd;
    xd += zd;
    *x = (int32_t)xi;
    *d = (int32_t)xd;
  };
  // rounds are counted from klo in every lane; a lane without a replay has klo == ka and idles
  // through the replay rounds of the others
  const bool any_warm = __builtin_amdgcn_ballot_w64(wact) != 0;
  const int32_t r_main = any_warm ? kSegWarm : 0;  // first round of the lanes' own pairs
  // (lanes without a replay: their pairs start at round r_main, so their words are fetched from klo - r_main)
  // -> give them a klo that makes round r_main their pair ka
  const int32_t klo_eff = wact ? klo : ka - r_main;
  auto fetch = [&](int32_t r) {  // the words of rounds [r, r + kLStage) (a lane without replay has no pairs before ka)
#pragma unroll
    for (int half = 0; half < 2; half++) {
      const int src = ((l >> 1) + 32 * half) << 2;
      const int32_t k0 = __builtin_amdgcn_ds_bpermute(src, klo_eff) + r + 4 * (l & 1);
      const int32_t lo_s = __builtin_amdgcn_ds_bpermute(src, klo);
      const int32_t ke_s = __builtin_amdgcn_ds_bpermute(src, ke);
      const int32_t pu_s = __builtin_amdgcn_ds_bpermute(src, Pu);
      const int64_t po = ((int64_t)__builtin_amdgcn_ds_bpermute(src, (int32_t)(pair_off >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int32_t)pair_off);
      const int32_t* yi = reinterpret_cast<const int32_t*>(in + po);
      const int32_t* yd = yi + pu_s;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const bool inb = k0 + q >= lo_s && k0 + q < ke_s;
        const int32_t a = inb ? yi[k0 + q] : 0, b = inb ? yd[k0 + q] : 0;
        if (half == 0) {
          ra[q] = a;
          rb[q] = b;
        } else {
          rc[q] = a;
          rd[q] = b;
        }
      }
    }
  };
  const int32_t n_rounds = r_main + __builtin_amdgcn_readfirstlane(wave_reduce(ke - ka, OpMax()));
  fetch(0);
  for (int32_t r = 0; r < n_rounds; r++) {
    if ((r & (kLStage - 1)) == 0) {
      stage();
      fetch(r + kLStage);
    }
    if (r == r_main && any_warm) {
      // the replay is over: everything before `own` is the predecessors'; the state from there goes to the check
      settle_upto(wact && !fail, own, false);
      dump_state(wact && !fail, dumpW, gi, own);
      if (!wact) zi = xi = zd = xd = 0;  // (idled through the replay rounds on zero words)
    }
    int32_t x, d;
    next_pair(r, &x, &d);
    if (r < r_main) round(warm_t, wact, x, d);
    else round(main_t, klo_eff + r < ke, x, d);
  }
  if (n_rounds == r_main && any_warm) {  // (no lane has pairs of its own: cannot happen for s > 0, kept for symmetry)
    settle_upto(wact && !fail, own, false);
    dump_state(wact && !fail, dumpW, gi, own);
  }
  // everything this segment owns becomes final; the state from `cap` on goes to the next segment's check
  const bool ok = sim && !fail;
  settle_upto(ok, lim_main, true);
  if (sim && fail) {
    if (atomicCAS(&units[sd.unit].fb, 0, 1) == 0) atomicAdd(nfail, 1);
    atomicAdd(nfail + 4, 1);
  }
  dump_state(ok && hasn, dumpT, gi + 1, cap);
}

}  // namespace cdcx
