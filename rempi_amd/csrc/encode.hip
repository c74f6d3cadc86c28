// encode.hip -- CDC record-side kernels for gfx950.
//
// Pipeline (one batch = many independent rank streams):
//   set discovery -> stable partition by table (T-order) -> length increments + prefix
//   -> chunk boundaries (A3) -> units -> per-unit compaction (A3 add) -> tile sort + merge
//   rank = clock order (A4) -> epoch line in libstdc++ hash order (A4) -> chain (A7)
//   -> edit-sequence positions + deltas (A8) -> sizes -> serialization with LP (A5, A6, A9,
//   A11) -> footer (A12).
// Integer/byte work only: HBM-bound passes are written for coalesced 16-byte accesses,
// no MFMA.
#include <hip/hip_runtime.h>

#include "cdcx_device.h"
#include "cdcx_kernels.h"
#include "hash_order.h"

namespace cdcx {

// ---------------------------------------------------------------------------------------
// Set discovery + per-tile histograms in one pass over the records: hist[tile][set id]
// (bit 31: the tile's last record of that set is a matched event -- what the first record of
// the set in a later tile needs to know to tell whether it starts a new unmatched run) and,
// per rank, which matching_set_ids occur (limit: [0, kMaxSets)).
__global__ void __launch_bounds__(256) k_tile_hist(const int32_t* __restrict__ rec, const Tile* __restrict__ tiles,
                                                   uint32_t* __restrict__ hist, uint32_t* __restrict__ presence,
                                                   uint32_t* err) {
  // A rank has a handful of sets, so the 64 lanes of an LDS atomic mostly meet on one address
  // and are served one after the other.  Four copies of the two tables, picked by lane % 4 and
  // one bank apart, cut that to sixteen lanes per address; the copies are merged at the end.
  // (Eight copies are faster alone and slower beside the other lanes' kernels: LDS is what the
  // kernels of a busy GPU run short of first.)
  constexpr int kCopies = 4, kStride = kMaxSets + 1;
  __shared__ uint32_t h[kCopies * kStride];
  __shared__ uint32_t last[kCopies * kStride];  // max over the set's records of (index in tile + 1) << 1 | matched
  for (int q = threadIdx.x; q < kCopies * kStride; q += 256) {
    h[q] = 0;
    last[q] = 0;
  }
  __syncthreads();
  const Tile t = tiles[blockIdx.x];
  const int cp = (threadIdx.x & (kCopies - 1)) * kStride;
  // (all of the tile's loads are issued before the first atomic: one memory round trip per block)
  constexpr int PER = kTile / 256;
  int32_t sidv[PER], flv[PER];
#pragma unroll
  for (int q = 0; q < PER; q++) {
    const int i = q * 256 + threadIdx.x;
    const int32_t* rp = rec + (t.start + min(i, t.len - 1)) * 8;  // (rows past the tile's end re-read its last record)
    sidv[q] = t.len > 0 ? rp[7] : 0;
    flv[q] = t.len > 0 ? rp[2] : 0;
  }
#pragma unroll
  for (int q = 0; q < PER; q++) {
    const int i = q * 256 + threadIdx.x;
    if (i >= t.len) break;
    const int32_t sid = sidv[q];
    if ((uint32_t)sid >= (uint32_t)kMaxSets) raise_error(err, kErrLimit);
    else {
      atomicAdd(&h[cp + sid], 1u);
      atomicMax(&last[cp + sid], ((uint32_t)(i + 1) << 1) | (flv[q] == 1 ? 1u : 0u));
    }
  }
  __syncthreads();
  uint32_t v = 0, lm = 0;
#pragma unroll
  for (int q = 0; q < kCopies; q++) {
    v += h[q * kStride + threadIdx.x];
    lm = max(lm, last[q * kStride + threadIdx.x]);
  }
  hist[(int64_t)blockIdx.x * kMaxSets + threadIdx.x] = v | ((lm & 1u) << 31);
  const uint64_t nz = __builtin_amdgcn_ballot_w64(v != 0);
  if (lane_id() == 0 && (uint32_t)nz) atomicOr(&presence[t.rank * (kMaxSets / 32) + wave_id() * 2], (uint32_t)nz);
  if (lane_id() == 32 && (uint32_t)(nz >> 32)) atomicOr(&presence[t.rank * (kMaxSets / 32) + wave_id() * 2 + 1], (uint32_t)(nz >> 32));
}

// Dense table index per (rank, set id): tables are numbered in ascending set id, which is
// the order test_tables_map (a std::map) emits them in (rempi_encoder_cdc.cpp:785-800).
__global__ void __launch_bounds__(kMaxSets) k_set_dense(const uint32_t* __restrict__ presence, int16_t* __restrict__ dense,
                                                        int32_t* __restrict__ setlist, int32_t* __restrict__ nsets) {
  latency_kernel();
  const int r = blockIdx.x, sid = threadIdx.x;
  const uint32_t* p = presence + r * (kMaxSets / 32);
  const int w = sid >> 5, b = sid & 31;
  int below = __popc(p[w] & ((1u << b) - 1));
  for (int i = 0; i < w; i++) below += __popc(p[i]);
  const bool here = (p[w] >> b) & 1;
  dense[r * kMaxSets + sid] = here ? (int16_t)below : (int16_t)-1;
  if (here) setlist[r * kMaxSets + below] = sid;
  if (sid == kMaxSets - 1) nsets[r] = below + (here ? 1 : 0);
}

// Per rank: exclusive scan of the tile histograms in (table, tile) order -> where each
// tile's records of each table start in T-order; table starts; and for every (tile, table)
// what the table's last record before the tile was: prevm = 0 none, 1 unmatched, 3 matched.
__global__ void __launch_bounds__(256) k_hist_scan(const uint32_t* __restrict__ hist, const int32_t* __restrict__ tile0,
                                                   const int32_t* __restrict__ ntiles, const int32_t* __restrict__ nsets,
                                                   const int32_t* __restrict__ setlist, int32_t* __restrict__ base,
                                                   int32_t* __restrict__ tstart, uint8_t* __restrict__ prevm) {
  latency_kernel();
  __shared__ int32_t lds[4];
  const int r = blockIdx.x;
  const int T = nsets[r], t0 = tile0[r], nt = ntiles[r];
  int32_t run = 0;
  for (int t = 0; t < T; t++) {
    const int sid = setlist[r * kMaxSets + t];
    if (threadIdx.x == 0) tstart[r * (kMaxSets + 1) + t] = run;
    int32_t carry = 0;  // (tile + 1) << 2 | flags of the table's latest non-empty tile so far
    for (int c = 0; c < nt; c += 256) {
      int i = c + threadIdx.x;
      const uint32_t hv = (i < nt) ? hist[(int64_t)(t0 + i) * kMaxSets + sid] : 0u;
      const int32_t v = (int32_t)(hv & 0x7fffffffu);
      int32_t tot;
      int32_t ex = block_exclusive_scan<256>(v, 0, OpAdd(), lds, &tot);
      const int32_t f = v ? (((i + 1) << 2) | 1 | (int32_t)((hv >> 31) << 1)) : 0;
      int32_t ftot;
      const int32_t fex = max(carry, block_exclusive_scan<256>(f, 0, OpMax(), lds, &ftot));
      if (i < nt) {
        base[(int64_t)(t0 + i) * kMaxSets + t] = run + ex;
        prevm[(int64_t)(t0 + i) * kMaxSets + t] = (uint8_t)(fex & 3);
      }
      run += tot;
      carry = max(carry, ftot);
    }
  }
  if (threadIdx.x == 0) tstart[r * (kMaxSets + 1) + T] = run;
}

// Stable scatter of records into T-order.  Rounds of 256 consecutive records; within a
// wave, records with the same table find each other with one ballot per bit of the rank's
// table indexes, which keeps the partition stable for any number of tables.
//
// The same pass forms inc0, the length increment of each record if chunks were infinite
// (add(), :189-212): 1 for a matched event, 1 for an unmatched event that starts a new run of
// its table (the table's previous record is a matched event, or there is none), else 0.  The
// previous record of the table is a lower lane of the wave, or the last one of an earlier
// (round, wave) slot of the tile (carried through the slot scan), or the last one before the
// tile (prevm).  inc0s is laid out per tile (tile * kTile + index), so a rank's flags are
// contiguous from a kTile-aligned start; tsum = the tile's sum.  A record's stream position
// travels in its T-order record (TRec::info), which the chunk and unit searches read.
__global__ void __launch_bounds__(256, 8) k_scatter(const int32_t* __restrict__ rec, const Tile* __restrict__ tiles,
                                                 const int16_t* __restrict__ dense, const int32_t* __restrict__ base,
                                                 const uint8_t* __restrict__ prevm, const int32_t* __restrict__ nsets,
                                                 const int64_t* __restrict__ rec_off, TRec* __restrict__ trec,
                                                 uint8_t* __restrict__ inc0s, int32_t* __restrict__ tsum) {
  constexpr int ROUNDS = kTile / 256;
  // [round][wave][table]: count (then the count before the slot) | last record's flags << 12; half words,
  // since LDS is what the kernels of a busy GPU run short of first
  __shared__ uint16_t wc[ROUNDS * 4 * kMaxSets];
  static_assert(kTile < (1 << 12), "a tile's count must fit the low 12 bits");
  __shared__ int32_t lds[4];
  __shared__ uint8_t incs[kTile];  // the tile's flags, gathered so that a thread stores four consecutive ones
  for (int i = threadIdx.x; i < ROUNDS * 4 * kMaxSets / 2; i += 256) reinterpret_cast<uint32_t*>(wc)[i] = 0;
  const Tile t = tiles[blockIdx.x];
  const int w = wave_id(), l = lane_id();
  const uint64_t lt_mask = (l == 0) ? 0ull : (~0ull >> (64 - l));
  const int T = nsets[t.rank];
  const int tbits = T > 1 ? 32 - __clz(T - 1) : 0;  // bits of a table index of this rank
  int4 lo[ROUNDS], hi[ROUNDS];
#pragma unroll
  for (int j = 0; j < ROUNDS; j++) {
    const int i = j * 256 + threadIdx.x;
    if (i < t.len) {
      const int4* rp = reinterpret_cast<const int4*>(rec + (t.start + i) * 8);
      lo[j] = rp[0];
      hi[j] = rp[1];
    } else {
      lo[j] = make_int4(0, 0, 0, 0);
      hi[j] = make_int4(0, 0, 0, 0);
    }
  }
  __syncthreads();
  int my_t[ROUNDS];
  int my_rank[ROUNDS];
  int my_prev[ROUNDS];  // flags of the table's previous record when it is a lower lane of this wave, else 0
#pragma unroll
  for (int j = 0; j < ROUNDS; j++) {
    const int i = j * 256 + threadIdx.x;
    const bool valid = i < t.len;
    const int32_t sid = hi[j].w;
    const int tb = valid ? dense[t.rank * kMaxSets + ((uint32_t)sid < (uint32_t)kMaxSets ? sid : 0)] : 0;
    uint64_t peers = __builtin_amdgcn_ballot_w64(valid);
    for (int b = 0; b < tbits; b++) {
      uint64_t m = __builtin_amdgcn_ballot_w64(((tb >> b) & 1) != 0);
      peers &= ((tb >> b) & 1) ? m : ~m;
    }
    const uint64_t mm = __builtin_amdgcn_ballot_w64(valid && lo[j].z == 1);
    const uint64_t lower = peers & lt_mask;
    my_t[j] = tb;
    my_rank[j] = __popcll(lower);
    my_prev[j] = lower ? (1 | (int)(((mm >> (63 - __clzll((long long)lower))) & 1) << 1)) : 0;
    if (valid && lower == 0)
      wc[(j * 4 + w) * kMaxSets + tb] =
          (uint16_t)(__popcll(peers) | ((1 | (int)(((mm >> (63 - __clzll((long long)peers))) & 1) << 1)) << 12));
  }
  __syncthreads();
  if ((int)threadIdx.x < T) {  // exclusive scan over (round, wave) for each table: thread = table
    const int tb = threadIdx.x;
    int32_t run = 0;
    int32_t pf = prevm[(int64_t)blockIdx.x * kMaxSets + tb];
    for (int k = 0; k < ROUNDS * 4; k++) {
      const int32_t v = wc[k * kMaxSets + tb];
      wc[k * kMaxSets + tb] = (uint16_t)(run | (pf << 12));
      run += v & 0xfff;
      if (v >> 12) pf = v >> 12;
    }
  }
  __syncthreads();
  const int64_t rb = rec_off[t.rank];
  const int32_t spos0 = (int32_t)(t.start - rb);
  // (block-uniform bases + unsigned 32-bit indices: scalar base plus vector offset addressing)
  TRec* const trec_r = trec + rb;
  const int32_t* const base_b = base + (int64_t)blockIdx.x * kMaxSets;
  int32_t sum = 0;
#pragma unroll
  for (int j = 0; j < ROUNDS; j++) {
    const int i = j * 256 + threadIdx.x;
    if (i >= t.len) continue;
    const int tb = my_t[j];
    const int32_t slot = wc[(j * 4 + w) * kMaxSets + tb];
    const uint32_t pos = (uint32_t)(base_b[(uint32_t)tb] + (slot & 0xfff) + my_rank[j]);
    // lo = {count, type, flag, rank}, hi = {with_next, index, clock, set}
    TRec o;
    const bool matched = (lo[j].z == 1);
    o.src = lo[j].w;
    o.clk = hi[j].z;
    o.x = matched ? hi[j].y : lo[j].x;
    o.info = (matched ? (kInfoMatched | (hi[j].x != 0 ? kInfoWithNext : 0u)) : 0u) | (uint32_t)(spos0 + i);
    trec_r[pos] = o;
    const int prev = my_prev[j] ? my_prev[j] : (slot >> 12);
    const int32_t inc = (matched || prev != 1) ? 1 : 0;
    incs[i] = (uint8_t)inc;
    sum += inc;
  }
  sum = block_sum<256>(sum, lds);  // (barriers: incs is complete)
  if (threadIdx.x == 0) tsum[blockIdx.x] = sum;
  // (flags past the tile's length are never read)
  reinterpret_cast<uint32_t*>(inc0s + (int64_t)blockIdx.x * kTile)[threadIdx.x] =
      reinterpret_cast<const uint32_t*>(incs)[threadIdx.x];
}

// Per rank: exclusive scan of the tile sums of inc0 (toff) and their total (rtot).
__global__ void __launch_bounds__(256) k_rank_scan(const int32_t* __restrict__ tsum, const int32_t* __restrict__ tile0,
                                                   const int32_t* __restrict__ ntiles, int32_t* __restrict__ toff,
                                                   int32_t* __restrict__ rtot) {
  latency_kernel();
  __shared__ int32_t lds[4];
  const int r = blockIdx.x;
  const int t0 = tile0[r], nt = ntiles[r];
  int32_t run = 0;
  for (int c = 0; c < nt; c += 256) {
    int i = c + threadIdx.x;
    int32_t v = (i < nt) ? tsum[t0 + i] : 0, tot;
    int32_t ex = block_exclusive_scan<256>(v, 0, OpAdd(), lds, &tot);
    if (i < nt) toff[t0 + i] = run + ex;
    run += tot;
  }
  if (threadIdx.x == 0) rtot[r] = run;
}

// Chunk boundaries, one wave per rank (extract_encoder_input_format_chunk, :740-778):
// a chunk starting at s ends at the first e with L(s,e) > REMPI_MAX and with_next(e) == 0,
// or at the end of the stream.  L(s,e) = p0(e+1)-p0(s) + #tables whose first record in
// [s,e] is an unmatched run continuation (inc0 == 0; inside the chunk it starts a run),
// p0(x) = sum of inc0 over stream positions < x.
//
// p0 is never materialised: at a tile boundary it is the tile offset (toff), inside a tile
// the wave adds the flags before x (16 bytes per lane).  The search for e first walks tile
// boundaries (tile offsets only), then the one tile that holds the crossing, from registers.
__global__ void __launch_bounds__(64) k_chunks(const int32_t* __restrict__ rec, const int64_t* __restrict__ rec_off,
                                               const int64_t* __restrict__ nrec, const int32_t* __restrict__ toff,
                                               const int32_t* __restrict__ rtot, const int32_t* __restrict__ tile0,
                                               const uint8_t* __restrict__ inc0s, const TRec* __restrict__ trec,
                                               const int32_t* __restrict__ tstart, const int32_t* __restrict__ nsets,
                                               const int64_t* __restrict__ ccap_off, int64_t max_len,
                                               int2* __restrict__ chunks, int32_t* __restrict__ nchunks) {
  latency_kernel();
  const int r = blockIdx.x, l = lane_id();
  const int64_t rb = rec_off[r];
  const int32_t n = (int32_t)nrec[r];
  const int32_t t0 = tile0[r], nt = (n + kTile - 1) / kTile;
  const int T = nsets[r];
  const int32_t* ts = tstart + r * (kMaxSets + 1);
  const uint8_t* ib = inc0s + (int64_t)t0 * kTile;  // the rank's flags by stream position
  const int32_t total = rtot[r];
  // flags (0/1 bytes) among the first nb of a lane's 16 bytes
  auto count16 = [](uint4 v, int32_t nb) -> int32_t {
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
    int32_t c = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int32_t k = min(max(nb - 4 * q, 0), 4);
      c += __popc(wv[q] & (k == 4 ? 0xffffffffu : ((1u << (8 * k)) - 1u)));
    }
    return c;
  };
  auto P = [&](int32_t x) -> int32_t {  // p0(x), 0 <= x <= n
    const int32_t q = x >> 10, wq = x & (kTile - 1);
    int32_t v = q < nt ? toff[t0 + q] : total;
    if (wq) {
      const int32_t nb = min(max(wq - 16 * l, 0), 16);
      const int32_t c = nb ? count16(*reinterpret_cast<const uint4*>(ib + (int64_t)q * kTile + 16 * l), nb) : 0;
      v += wave_reduce(c, OpAdd());
    }
    return v;
  };
  static_assert(kTile == 1024, "a tile's flags are 16 bytes per lane of one wave");
  int32_t s = 0, k = 0, p0s = 0;
  while (s < n) {
    int32_t corr[kMaxSets / 64];  // first-in-chunk unmatched continuation positions
#pragma unroll
    for (int q = 0; q < kMaxSets / 64; q++) {
      const int tb = q * 64 + l;
      corr[q] = INT32_MAX;
      if (tb < T) {
        int32_t lo = ts[tb], hi = ts[tb + 1];
        while (lo < hi) {
          int32_t mid = (lo + hi) >> 1;
          if ((int32_t)(trec[rb + mid].info & kInfoPos) < s) lo = mid + 1; else hi = mid;
        }
        if (lo < ts[tb + 1]) {
          int32_t f = (int32_t)(trec[rb + lo].info & kInfoPos);
          if (ib[f] == 0) corr[q] = f;
        }
      }
    }
    auto L = [&](int32_t e, int32_t p_next) -> int64_t {  // p_next = p0(e + 1)
      int c = 0;
#pragma unroll
      for (int q = 0; q < kMaxSets / 64; q++) c += (corr[q] <= e) ? 1 : 0;
      c = wave_reduce(c, OpAdd());
      return (int64_t)(p_next - p0s) + c;
    };
    int32_t e;
    if (L(n - 1, total) <= max_len) {
      e = n - 1;
    } else {
      // smallest tile boundary b in ((s >> 10), nt] with L(min(b * kTile, n) - 1) > max_len
      int32_t lo = (s >> 10) + 1, hi = nt;
      while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;  // < nt: the boundary lies inside the stream
        if (L(mid * kTile - 1, toff[t0 + mid]) > max_len) hi = mid; else lo = mid + 1;
      }
      // the crossing lies in tile lo - 1: its flags, a lane's sum, the sums of the lanes before
      const int32_t q = lo - 1;
      const uint4 v = *reinterpret_cast<const uint4*>(ib + (int64_t)q * kTile + 16 * l);
      const int32_t mine = count16(v, min(max(min(kTile, n - q * kTile) - 16 * l, 0), 16));
      const int32_t pre = wave_inclusive_scan(mine, OpAdd()) - mine;
      const int32_t tb0 = toff[t0 + q];
      auto Pt = [&](int32_t wq) -> int32_t {  // p0(q * kTile + wq), 1 <= wq <= kTile
        const int32_t ln = __builtin_amdgcn_readfirstlane((wq - 1) >> 4);
        const uint4 u = make_uint4(__builtin_amdgcn_readlane(v.x, ln), __builtin_amdgcn_readlane(v.y, ln),
                                   __builtin_amdgcn_readlane(v.z, ln), __builtin_amdgcn_readlane(v.w, ln));
        return tb0 + __builtin_amdgcn_readlane(pre, ln) + count16(u, wq - 16 * ln);
      };
      int32_t xlo = max(s, q * kTile) + 1, xhi = min(lo * kTile, n);  // e + 1 in [xlo, xhi]; L(xhi - 1) > max_len
      while (xlo < xhi) {
        const int32_t xm = (xlo + xhi) >> 1;
        if (L(xm - 1, Pt(xm - q * kTile)) > max_len) xhi = xm; else xlo = xm + 1;
      }
      e = xlo - 1;
      while (e < n - 1 && rec[(rb + e) * 8 + 4] != 0) e++;
    }
    if (l == 0) chunks[ccap_off[r] + k] = make_int2(s, e);
    k++;
    s = e + 1;
    if (s < n) p0s = P(s);
  }
  if (l == 0) nchunks[r] = k;
}

// For every (chunk, table): the table's T-order sub-range that falls inside the chunk; per
// chunk the number of non-empty tables (its units) and the sum of their lengths + 1.
__global__ void __launch_bounds__(kMaxSets) k_units_lb(const Chunk* __restrict__ ch, int32_t n_chunks,
                                                       const int64_t* __restrict__ lb_off, const int32_t* __restrict__ nsets,
                                                       const int32_t* __restrict__ tstart, const int64_t* __restrict__ rec_off,
                                                       const TRec* __restrict__ trec, int2* __restrict__ lohi,
                                                       int32_t* __restrict__ ucnt, int64_t* __restrict__ uw) {
  latency_kernel();
  __shared__ int64_t lds[kMaxSets / kWave];
  const int c = blockIdx.x;
  if (c >= n_chunks) return;
  const Chunk C = ch[c];
  const int T = nsets[C.rank];
  const int64_t rb = rec_off[C.rank];
  const int32_t* ts = tstart + C.rank * (kMaxSets + 1);
  const int tb = threadIdx.x;
  int64_t mine = 0;
  if (tb < T) {
    int32_t r0 = ts[tb], r1 = ts[tb + 1];
    auto lb = [&](int32_t x) {
      int32_t lo = r0, hi = r1;
      while (lo < hi) {
        int32_t mid = (lo + hi) >> 1;
        if ((int32_t)(trec[rb + mid].info & kInfoPos) < x) lo = mid + 1; else hi = mid;
      }
      return lo;
    };
    const int2 lh = make_int2(lb(C.s), lb(C.e + 1));
    lohi[lb_off[c] + tb] = lh;
    if (lh.y > lh.x) mine = ((int64_t)1 << 40) + (lh.y - lh.x) + 1;
  }
  const int64_t tot = block_sum<kMaxSets>(mine, lds);
  if (threadIdx.x == 0) {
    ucnt[c] = (int32_t)(tot >> 40);
    uw[c] = tot & (((int64_t)1 << 40) - 1);
  }
}

// ---------------------------------------------------------------------------------------
// Per-unit compaction (add(), :178-218): matched keys/indices in observed order, the
// with_previous list, unmatched runs (merged while no matched event of the table
// intervenes) -> counts M, U, W.
__global__ void __launch_bounds__(256) k_unit_prep(Unit* __restrict__ units, const TRec* __restrict__ trec,
                                                   uint64_t* __restrict__ mkey, int32_t* __restrict__ midx,
                                                   int32_t* __restrict__ wp, int32_t* __restrict__ run_id,
                                                   uint64_t* __restrict__ run_cnt, uint32_t* err) {
  // The three counts (matched, with_next, unmatched run starts) travel through one scan,
  // packed into 21-bit fields.
  __shared__ uint64_t lds[4];
  Unit& u = units[blockIdx.x];
  const int64_t a = u.a;
  const int32_t n = u.n;
  int32_t cm = 0, cw = 0, cr = 0;
  constexpr uint64_t F = 1ull << 21;
  for (int32_t b = 0; b < n; b += 256) {
    const int32_t k = b + threadIdx.x;
    const bool valid = k < n;
    const TRec r = valid ? trec[a + k] : TRec{0, 0, 0, 0};
    const bool m = valid && (r.info >> 31);
    const bool wn = m && (r.info & kInfoWithNext);
    const bool rs = valid && !m && ((k == 0) || (trec[a + k - 1].info >> 31));
    uint64_t tot;
    const uint64_t ex =
        block_exclusive_scan<256>((uint64_t)m + (uint64_t)wn * F + (uint64_t)rs * F * F, (uint64_t)0, OpAdd(), lds, &tot);
    const int32_t mo = cm + (int32_t)(ex & (F - 1));
    if (m) {
      mkey[a + mo] = pack_key(r.clk, r.src);
      midx[a + mo] = r.x;
    }
    if (wn) wp[a + cw + (int32_t)((ex >> 21) & (F - 1))] = mo;
    if (rs) {  // the run: this and the following unmatched records (add(), :205-208)
      uint64_t cnt = sext(r.x);
      for (int32_t j = k + 1; j < n; j++) {
        const TRec q = trec[a + j];
        if (q.info >> 31) break;
        cnt += sext(q.x);
      }
      const int32_t ro = cr + (int32_t)(ex >> 42);
      run_id[a + ro] = mo;
      run_cnt[a + ro] = cnt;
    }
    cm += (int32_t)(tot & (F - 1));
    cw += (int32_t)((tot >> 21) & (F - 1));
    cr += (int32_t)(tot >> 42);
  }
  if (threadIdx.x == 0) {
    u.M = cm;
    u.U = cr;
    u.W = cw;
  }
  // A table must not end inside a with_next group (format(), :229-233).
  __syncthreads();
  if (threadIdx.x == 0 && cw > 0 && wp[a + cw - 1] == cm - 1) raise_error(err, kErrTruncated);
}

// ---------------------------------------------------------------------------------------
// Clock order (format(), :235-239), windowed.  Traces arrive nearly in clock order: an
// event's rank in its unit differs from its observed index by a few dozen at most.  If every
// pair q < p with D < p - q <= 2D + 1 has key[q] <= key[p], then (by induction on p - q,
// stepping D + 1 at a time) every pair more than D apart is in order, so
//   rank(p) = #{q < p - D} + #{q in [p - D, p + D] ordered before p}
//           = p - D + (window count, with key 0 standing in for positions before the unit
//                      and ~0 for those after it)
// where "ordered before" is (key, index) order.  One pass, no sort: each tile of 1024 events
// loads its events plus a halo of 2D + 1 before and D after, checks the condition for its
// events (a key equal to the ~0 sentinel fails it too) and writes cord / inv / skey.  The cost
// is linear in D, so every unit first tries D = 40 and only a unit with a failing tile repeats
// with D = kRankWin.  A unit that fails that too is flagged (Unit::wfail = 1); the host ranks
// it again with the tile sort below, launched over the flagged units' tiles only.
namespace {
// One attempt with window D.  Returns (to every thread) whether the condition failed for any
// event of the tile; the ranks of the tile are left in rk[] and own[] holds the thread's keys.
template <int D>
__device__ __forceinline__ bool window_rank_try(const Unit& u, int32_t t0, int len, const uint64_t* __restrict__ mkey,
                                                uint64_t* xk, int32_t* rk, uint64_t (&own)[4]) {
  constexpr int H = 2 * D + 1;  // halo before the tile
  constexpr int NX = H + kSortTile + D;
  static_assert(D % 4 == 0 && D >= 8, "bulk loops run D - 4 iterations, unrolled by 4");
  // Key k of the tile's range sits at xk[k + k / 4]: a thread reads keys 4t + x, and the pad
  // turns its 32 B lane stride into 40 B (10 banks), so 32 lanes read distinct banks.
  for (int k = threadIdx.x; k < NX; k += 256) {
    const int32_t q = t0 - H + k;
    xk[k + (k >> 2)] = q < 0 ? 0ull : (q >= u.M ? ~0ull : mkey[u.a + q]);
  }
  __syncthreads();
  const int L = 4 * threadIdx.x;  // own events: tile offsets L..L+3 = keys L + H + j
  const uint64_t* x0 = xk + 5 * threadIdx.x;
  auto key = [&](int x) { return x0[x + (x >> 2)]; };  // key L + x (x >= 0)
#pragma unroll
  for (int j = 0; j < 4; j++) own[j] = key(H + j);
  // check: event j's window is keys L + j .. L + j + D (positions p - 2D - 1 .. p - D - 1);
  // x = 3 .. D lies in all four.  (Loops stay rolled: fully unrolled, the compiler keeps
  // the whole window in registers and the kernel runs at 2 waves/SIMD.)
  uint64_t mc = max(key(3), key(D));
#pragma unroll 4
  for (int x = 4; x < D; x++) mc = max(mc, key(x));
  bool bad = false;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    uint64_t m = mc;
#pragma unroll
    for (int x = j; x < 3; x++) m = max(m, key(x));
#pragma unroll
    for (int x = D + 1; x <= D + j; x++) m = max(m, key(x));
    bad |= (L + j < len) && (m > own[j] || own[j] == ~0ull);
  }
  // count: event j's window is keys L + H + j - D .. L + H + j + D; earlier positions count
  // when key <= own (equal keys keep row order), later ones when key < own.  x = H - D + 3
  // .. H - 1 is before and inside all four windows, x = H + 4 .. H + D after and inside.
  int32_t cnt[4] = {0, 0, 0, 0};
#pragma unroll 4
  for (int x = H - D + 4; x < H; x++) {
    const uint64_t v = key(x);
#pragma unroll
    for (int j = 0; j < 4; j++) cnt[j] += v <= own[j] ? 1 : 0;
  }
#pragma unroll 4
  for (int x = H + 4; x < H + D; x++) {
    const uint64_t v = key(x);
#pragma unroll
    for (int j = 0; j < 4; j++) cnt[j] += v < own[j] ? 1 : 0;
  }
#pragma unroll
  for (int e = 0; e < 4; e++) {  // key H - D + e: inside the windows of events j <= e
    const uint64_t v = key(H - D + e);
#pragma unroll
    for (int j = 0; j <= e; j++) cnt[j] += v <= own[j] ? 1 : 0;
  }
#pragma unroll
  for (int e = 0; e < 4; e++) {  // the own events among themselves
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (j > e) cnt[j] += own[e] <= own[j] ? 1 : 0;
      if (j < e) cnt[j] += own[e] < own[j] ? 1 : 0;
    }
  }
#pragma unroll
  for (int e = 0; e <= 3; e++) {  // key H + D + e: inside the windows of events j >= e
    const uint64_t v = key(H + D + e);
#pragma unroll
    for (int j = e; j < 4; j++) cnt[j] += v < own[j] ? 1 : 0;
  }
  __syncthreads();  // (rk shares its storage with xk: every thread is done with the keys)
#pragma unroll
  for (int j = 0; j < 4; j++) rk[L + j] = t0 + L + j - D + cnt[j];
  return __syncthreads_or(bad);
}
}  // namespace

namespace {
// Ranks one tile with window D and writes cord / inv / skey; returns whether the condition
// failed for any of its events (then what it wrote is not to be used).
template <int D>
__device__ __forceinline__ bool window_rank_tile(const Unit& u, int32_t tile, const uint64_t* __restrict__ mkey,
                                                 int32_t* __restrict__ cord, int32_t* __restrict__ inv,
                                                 uint64_t* __restrict__ skey, uint64_t* xk, int32_t* rk) {
  const int32_t t0 = tile * kSortTile;
  const int len = min(kSortTile, u.M - t0);
  uint64_t own[4];
  const bool bad = window_rank_try<D>(u, t0, len, mkey, xk, rk, own);
  const int L = 4 * threadIdx.x;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    if (L + j < len) {
      const int32_t r = rk[L + j];
      inv[u.a + r] = t0 + L + j;
      skey[u.key_off + r] = key_words(own[j]);
    }
  }
  for (int k = threadIdx.x; k < len; k += 256) cord[u.a + t0 + k] = rk[k];
  return bad;
}
// (the bench traces: the farthest pair out of clock order in a unit is 31-37 places apart)
constexpr int kRankNarrow = 40;
}  // namespace

// First attempt, one block per tile, narrow window.  A remote violation can change the rank
// of an event whose own neighbourhood is in order, so a failing tile sends its whole unit to
// the wide window (Unit::wfail bit 2).
__global__ void __launch_bounds__(256) k_window_rank(Unit* __restrict__ units, const SortTile* __restrict__ st,
                                                     const uint64_t* __restrict__ mkey, int32_t* __restrict__ cord,
                                                     int32_t* __restrict__ inv, uint64_t* __restrict__ skey) {
  constexpr int NX = 2 * kRankNarrow + 1 + kSortTile + kRankNarrow;
  __shared__ uint64_t xk[NX + NX / 4 + 1];
  int32_t* rk = reinterpret_cast<int32_t*>(xk);  // the tile's ranks, once the keys are no longer needed
  static_assert(sizeof(xk) >= kSortTile * sizeof(int32_t), "the ranks fit the key storage");
  const SortTile w = st[blockIdx.x];
  if (w.unit < 0) return;  // past the batch's sort tiles (the grid is an upper bound)
  const Unit u = units[w.unit];
  if (window_rank_tile<kRankNarrow>(u, w.tile, mkey, cord, inv, skey, xk, rk) && threadIdx.x == 0)
    atomicOr(&units[w.unit].wfail, 4);
}

// Second attempt, one block per unit that the narrow window could not rank: all its tiles
// again with D = kRankWin.  A unit that fails here too keeps wfail bit 0 for the tile sort.
__global__ void __launch_bounds__(256) k_window_rank_wide(Unit* __restrict__ units, const uint64_t* __restrict__ mkey,
                                                          int32_t* __restrict__ cord, int32_t* __restrict__ inv,
                                                          uint64_t* __restrict__ skey) {
  constexpr int NX = 2 * kRankWin + 1 + kSortTile + kRankWin;
  __shared__ uint64_t xk[NX + NX / 4 + 1];
  int32_t* rk = reinterpret_cast<int32_t*>(xk);  // the tile's ranks, once the keys are no longer needed
  const Unit u = units[blockIdx.x];
  if (!(u.wfail & 4)) return;
  bool bad = false;
  for (int32_t tile = 0; tile * kSortTile < u.M; tile++) {
    bad |= window_rank_tile<kRankWin>(u, tile, mkey, cord, inv, skey, xk, rk);
    __syncthreads();  // rk and xk are reused by the next tile
  }
  if (threadIdx.x == 0) units[blockIdx.x].wfail = bad ? 1 : 0;
}

// ---------------------------------------------------------------------------------------
// Clock order (format(), :235-239).  Sort tiles of <= 1024 matched events in LDS by
// (key, observed index); then every event's global rank = its rank in its own tile + the
// number of smaller events in the unit's other tiles (tile min/max prune, binary search
// where ranges overlap).  Near-sorted traces overlap only with neighbour tiles.
__global__ void __launch_bounds__(256) k_sort_tiles(const Unit* __restrict__ units, const SortTile* __restrict__ st,
                                                    const uint64_t* __restrict__ mkey, uint64_t* __restrict__ tkey,
                                                    int32_t* __restrict__ lrank, uint64_t* __restrict__ tminmax) {
  // Bitonic network held in registers: thread t owns elements 4t..4t+3.  Strides 1 and 2
  // compare inside a thread, strides 4..128 exchange with lane t ^ (stride/4) of the same
  // wave (shuffles), and only strides 256 and 512 (3 of the 55 stages) go through LDS.
  // Order: (key, original index), so equal keys keep row order.
  __shared__ uint64_t xk[kSortTile];
  __shared__ int32_t xi[kSortTile];
  const SortTile w = st[blockIdx.x];
  const Unit u = units[w.unit];
  const int64_t base = u.a + (int64_t)w.tile * kSortTile;
  const int len = min(kSortTile, u.M - w.tile * kSortTile);
  const int t = threadIdx.x;
  uint64_t vk[4];
  int32_t vi[4];
  auto gt = [](uint64_t ak, int32_t ai, uint64_t bk, int32_t bi) { return ak > bk || (ak == bk && ai > bi); };
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int e = 4 * t + q;
    vk[q] = (e < len) ? mkey[base + e] : ~0ull;
    vi[q] = e;
  }
  for (int size = 2; size <= kSortTile; size <<= 1) {
    const bool asc = ((4 * t) & size) == 0;  // the same for all four elements when size >= 4
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride >= 4) {
        uint64_t ok[4];
        int32_t oi[4];
        if (stride >= 256) {
#pragma unroll
          for (int q = 0; q < 4; q++) {
            xk[4 * t + q] = vk[q];
            xi[4 * t + q] = vi[q];
          }
          __syncthreads();
#pragma unroll
          for (int q = 0; q < 4; q++) {
            ok[q] = xk[(4 * t + q) ^ stride];
            oi[q] = xi[(4 * t + q) ^ stride];
          }
          __syncthreads();
        } else {
          const int sl = stride >> 2;
#pragma unroll
          for (int q = 0; q < 4; q++) {
            ok[q] = __shfl_xor(vk[q], sl, 64);
            oi[q] = __shfl_xor(vi[q], sl, 64);
          }
        }
        // keep the min when this element is the lower of an ascending pair or the upper of
        // a descending one
        const bool keep_min = (((4 * t) & stride) == 0) == asc;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          if (keep_min == gt(vk[q], vi[q], ok[q], oi[q])) {
            vk[q] = ok[q];
            vi[q] = oi[q];
          }
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; q++) {
          if (q & stride) continue;  // q is the lower element of the pair (q, q + stride)
          const bool a2 = (size == 2) ? (((4 * t + q) & 2) == 0) : asc;
          if (gt(vk[q], vi[q], vk[q + stride], vi[q + stride]) == a2) {
            const uint64_t tk = vk[q];
            const int32_t ti = vi[q];
            vk[q] = vk[q + stride];
            vi[q] = vi[q + stride];
            vk[q + stride] = tk;
            vi[q + stride] = ti;
          }
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int r = 4 * t + q;
    if (r < len) {
      tkey[base + r] = vk[q];
      lrank[base + vi[q]] = r;
    }
    if (r == 0) tminmax[2 * (u.sort_tile0 + w.tile)] = vk[q];
    if (r == len - 1) tminmax[2 * (u.sort_tile0 + w.tile) + 1] = vk[q];
  }
}

__global__ void __launch_bounds__(256) k_rank_tiles(const Unit* __restrict__ units, const SortTile* __restrict__ st,
                                                    const uint64_t* __restrict__ mkey, const uint64_t* __restrict__ tkey,
                                                    const int32_t* __restrict__ lrank, const uint64_t* __restrict__ tminmax,
                                                    int32_t* __restrict__ cord, int32_t* __restrict__ inv,
                                                    uint64_t* __restrict__ skey) {
  // Tile-level pruning first: tiles wholly below every key of this tile add their length,
  // tiles wholly above add nothing, and only the overlapping ones (for near-sorted traces
  // the neighbours) are binary-searched per key.
  constexpr int kMaxOv = 64;
  __shared__ int32_t ov[kMaxOv];
  __shared__ int32_t nov, below;
  const SortTile w = st[blockIdx.x];
  const Unit u = units[w.unit];
  const int nt = (u.M + kSortTile - 1) / kSortTile;
  const uint64_t* mm = tminmax + 2 * (int64_t)u.sort_tile0;
  const int len = min(kSortTile, u.M - w.tile * kSortTile);
  const uint64_t wmin = mm[2 * w.tile], wmax = mm[2 * w.tile + 1];
  if (threadIdx.x == 0) {
    nov = 0;
    below = 0;
  }
  __syncthreads();
  int32_t my_below = 0;
  for (int q = threadIdx.x; q < nt; q += 256) {
    if (q == w.tile) continue;
    const int qlen = min(kSortTile, u.M - q * kSortTile);
    const uint64_t qmin = mm[2 * q], qmax = mm[2 * q + 1];
    // q < w counts keys <= x (equal keys of earlier rows first), q > w keys < x
    const bool all = (q < w.tile) ? (qmax <= wmin) : (qmax < wmin);
    const bool none = (q < w.tile) ? (qmin > wmax) : (qmin >= wmax);
    if (all) my_below += qlen;
    else if (!none) {
      const int k = atomicAdd(&nov, 1);
      if (k < kMaxOv) ov[k] = q;
    }
  }
  my_below = wave_reduce(my_below, OpAdd());
  if (lane_id() == 0 && my_below) atomicAdd(&below, my_below);
  __syncthreads();
  const int n_ov = nov;
  const int32_t base = below;
  // the (usually two) overlapping neighbour tiles are searched in LDS
  constexpr int kLdsTiles = 2;
  __shared__ uint64_t nk[kLdsTiles][kSortTile];
  if (n_ov <= kLdsTiles) {
    for (int k = 0; k < n_ov; k++) {
      const int q = ov[k];
      const int qlen = min(kSortTile, u.M - q * kSortTile);
      for (int t = threadIdx.x; t < qlen; t += 256) nk[k][t] = tkey[u.a + (int64_t)q * kSortTile + t];
    }
    __syncthreads();
  }
  for (int j = threadIdx.x; j < len; j += 256) {
    const int32_t i = w.tile * kSortTile + j;
    const uint64_t x = mkey[u.a + i];
    int32_t rank = lrank[u.a + i] + base;
    if (n_ov <= kLdsTiles) {
      for (int k = 0; k < n_ov; k++) {
        const int q = ov[k];
        const int qlen = min(kSortTile, u.M - q * kSortTile);
        const uint64_t* tk = nk[k];
        int lo = 0, hi = qlen;
        if (q < w.tile) {
          while (lo < hi) { const int mid = (lo + hi) >> 1; if (tk[mid] <= x) lo = mid + 1; else hi = mid; }
        } else {
          while (lo < hi) { const int mid = (lo + hi) >> 1; if (tk[mid] < x) lo = mid + 1; else hi = mid; }
        }
        rank += lo;
      }
    } else if (n_ov <= kMaxOv) {
      for (int k = 0; k < n_ov; k++) {
        const int q = ov[k];
        const int qlen = min(kSortTile, u.M - q * kSortTile);
        const uint64_t* tk = tkey + u.a + (int64_t)q * kSortTile;
        int lo = 0, hi = qlen;
        if (q < w.tile) {
          while (lo < hi) { const int mid = (lo + hi) >> 1; if (tk[mid] <= x) lo = mid + 1; else hi = mid; }
        } else {
          while (lo < hi) { const int mid = (lo + hi) >> 1; if (tk[mid] < x) lo = mid + 1; else hi = mid; }
        }
        rank += lo;
      }
    } else {  // many overlapping tiles (e.g. a reversed or random permutation): test them all
      for (int q = 0; q < nt; q++) {
        if (q == w.tile) continue;
        const int qlen = min(kSortTile, u.M - q * kSortTile);
        const uint64_t qmin = mm[2 * q], qmax = mm[2 * q + 1];
        const bool all = (q < w.tile) ? (qmax <= wmin) : (qmax < wmin);
        const bool none = (q < w.tile) ? (qmin > wmax) : (qmin >= wmax);
        if (all || none) continue;  // already in base / contributes nothing
        const uint64_t* tk = tkey + u.a + (int64_t)q * kSortTile;
        int lo = 0, hi = qlen;
        if (q < w.tile) {
          while (lo < hi) { const int mid = (lo + hi) >> 1; if (tk[mid] <= x) lo = mid + 1; else hi = mid; }
        } else {
          while (lo < hi) { const int mid = (lo + hi) >> 1; if (tk[mid] < x) lo = mid + 1; else hi = mid; }
        }
        rank += lo;
      }
    }
    cord[u.a + i] = rank;
    inv[u.a + rank] = i;
    skey[u.key_off + rank] = key_words(x);
  }
}

// ---------------------------------------------------------------------------------------
// Epoch line (format(), :246-267): per source the last clock in sorted order, listed in
// the iteration order of the reference's unordered_map<size_t,size_t> fed in sorted
// order.  Also the clock-order check of :249-256 (equal (clock, source) keys, clock != 0).
//
// Two instances: HCAP = 512 (up to 256 distinct sources per table, 9 KB of LDS, so a CU
// runs 8 blocks) for every unit, and HCAP = 2 * kMaxUnitSources (72 KB of LDS) only for the
// units the small one marks with S = -1.
template <int HCAP>
__global__ void __launch_bounds__(256) k_epoch(Unit* __restrict__ units, const uint64_t* __restrict__ skey,
                                               uint64_t* __restrict__ ep_rank, uint64_t* __restrict__ ep_clk,
                                               int64_t ep_stride, uint32_t* err) {
  constexpr int LCAP = HCAP / 2;  // distinct sources this instance can list
  constexpr bool kBig = HCAP >= 2 * kMaxUnitSources;
  __shared__ int32_t hsrc[HCAP];
  __shared__ int32_t hpos[HCAP];
  __shared__ int32_t hclk[HCAP];
  __shared__ int32_t nlist;
  // After compaction the hash arrays are reused as the sort buffers and emulator storage.
  Unit& u = units[blockIdx.x];
  if (u.wfail != 0) return;  // not ranked yet (k_window_rank), or already done
  if (kBig && u.S != -1) return;
  const int64_t a = u.a, ka = u.key_off;
  const int64_t ea = epoch_slot(blockIdx.x, a, ep_stride);
  const int32_t M = u.M;
  for (int i = threadIdx.x; i < HCAP; i += 256) {
    hsrc[i] = INT32_MIN;
    hpos[i] = INT32_MAX;
    hclk[i] = INT32_MIN;
  }
  if (threadIdx.x == 0) nlist = 0;
  __syncthreads();
  for (int32_t r = threadIdx.x; r < M; r += 256) {
    const uint64_t k = key_words(skey[ka + r]);  // (skey holds {source, clock} words)
    const int32_t src = key_source(k), clk = key_clock(k);
    if (!kBig && r + 1 < M && key_words(skey[ka + r + 1]) == k && clk != 0) raise_error(err, kErrClockOrder);
    if (src == INT32_MIN) { raise_error(err, kErrLimit); continue; }
    uint32_t h = ((uint32_t)src * 2654435761u) % HCAP;
    for (int probe = 0; probe < HCAP; probe++) {
      int32_t old = atomicCAS(&hsrc[h], INT32_MIN, src);
      if (old == INT32_MIN || old == src) {
        atomicMin(&hpos[h], r);
        atomicMax(&hclk[h], clk);
        break;
      }
      h = (h + 1) % HCAP;
    }
  }
  __syncthreads();
  // Compact (src, first sorted position, last clock) triples.
  __shared__ int32_t lpos[LCAP];
  __shared__ int32_t lsrc[LCAP];
  __shared__ int32_t lclk[LCAP];
  for (int i = threadIdx.x; i < HCAP; i += 256) {
    if (hsrc[i] != INT32_MIN) {
      int q = atomicAdd(&nlist, 1);
      if (q < LCAP) {
        lpos[q] = hpos[i];
        lsrc[q] = hsrc[i];
        lclk[q] = hclk[i];
      }
    }
  }
  __syncthreads();
  const int S = nlist;
  if (S > LCAP) {
    if (threadIdx.x == 0) {
      if (kBig) {
        raise_error(err, kErrLimit);
        u.S = 0;
      } else {
        u.S = -1;  // more sources than the small table holds: the big instance redoes it
      }
    }
    return;
  }
  int P2 = 1;
  while (P2 < S) P2 <<= 1;
  for (int i = S + threadIdx.x; i < P2; i += 256) lpos[i] = INT32_MAX;
  __syncthreads();
  // Bitonic sort of the triples by first sorted position = unordered_map insertion order.
  for (int size = 2; size <= P2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int p = threadIdx.x; p < P2 / 2; p += 256) {
        const int i = 2 * p - (p & (stride - 1));
        const int j = i + stride;
        const bool up = ((i & size) == 0);
        if ((lpos[i] > lpos[j]) == up) {
          int32_t t0 = lpos[i]; lpos[i] = lpos[j]; lpos[j] = t0;
          t0 = lsrc[i]; lsrc[i] = lsrc[j]; lsrc[j] = t0;
          t0 = lclk[i]; lclk[i] = lclk[j]; lclk[j] = t0;
        }
      }
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) {
    uint64_t* hk = reinterpret_cast<uint64_t*>(hsrc);  // HCAP*4 bytes = kMaxUnitSources*8
    int32_t* hn = hpos;
    int32_t* hb = hclk;  // bucket array: capacity HCAP >= hash_bucket_capacity(2048)=2357?
    HashOrder ho;
    ho.init(hk, hn, hb);
    for (int q = 0; q < S; q++) ho.insert_new((uint64_t)(int64_t)lsrc[q]);
    int j = 0;
    for (int32_t p = ho.head; p != -1; p = ho.next[p], j++) {
      ep_rank[ea + j] = (uint64_t)(int64_t)lsrc[p];
      ep_clk[ea + j] = (uint64_t)(int64_t)lclk[p];
    }
    u.S = S;
  }
}

template __global__ void k_epoch<512>(Unit*, const uint64_t*, uint64_t*, uint64_t*, int64_t, uint32_t*);
template __global__ void k_epoch<2 * kMaxUnitSources>(Unit*, const uint64_t*, uint64_t*, uint64_t*, int64_t, uint32_t*);

// ---------------------------------------------------------------------------------------
// Edit-sequence positions (A8).  With chain rows r_1<..<r_K (columns col_k) and r_0 =
// col_0 = -1, gap k lists ADD(rows r_{k-1}+1..r_k-1), REMOVE(cols col_{k-1}+1..col_k-1),
// IGNORE(col_k).  Hence, with Kr(r) = #chain rows < r and Kc(j) = #chain cols < j:
//   ADD of off-chain row r    at r + colprev(r) + 1 - Kr(r)
//   REMOVE of off-chain col j at rnext(j) + j - Kc(j)
//   IGNORE of chain row r     at r + c[r] - Kr(r)
// where colprev = last chain column before row r, rnext = row of the next chain node
// after column j (M for the end).  seq[2a+pos] = partner position << 2 | type.
enum : uint32_t { kIgn = 0, kAdd = 1, kRem = 2 };

namespace {
// Block-wide exclusive scan of (count, max) pairs for 256 threads.
__device__ __forceinline__ int2 block_scan_cnt_max(int2 v, int2* lds, int2* total) {
  const int l = lane_id(), w = wave_id();
  int2 inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int32_t ox = __shfl_up(inc.x, d, 64), oy = __shfl_up(inc.y, d, 64);
    if (l >= d) {
      inc.x += ox;
      inc.y = max(inc.y, oy);
    }
  }
  if (l == 63) lds[w] = inc;
  __syncthreads();
  int2 pre = make_int2(0, INT32_MIN);
  for (int q = 0; q < w; q++) {
    pre.x += lds[q].x;
    pre.y = max(pre.y, lds[q].y);
  }
  int2 tot = pre;
  for (int q = w; q < 4; q++) {
    tot.x += lds[q].x;
    tot.y = max(tot.y, lds[q].y);
  }
  int32_t ex = __shfl_up(inc.x, 1, 64), ey = __shfl_up(inc.y, 1, 64);
  if (l == 0) {
    ex = 0;
    ey = INT32_MIN;
  }
  *total = tot;
  __syncthreads();
  return make_int2(pre.x + ex, max(pre.y, ey));
}
}  // namespace

// Rows pass (4 rows per thread per round): Kr = #chain rows before r, colprev = last chain
// column before r.  posA of the ADD of off-chain row r (see above) and crow[k] = row of the
// k-th chain node.
__global__ void __launch_bounds__(256) k_pos_rows(const Unit* __restrict__ units, const int32_t* __restrict__ cord,
                                                  const uint8_t* __restrict__ chain, int32_t* __restrict__ posA,
                                                  int32_t* __restrict__ crow) {
  __shared__ int2 lds[4];
  const Unit u = units[blockIdx.x];
  const int64_t a = u.a;
  const int32_t M = u.M;
  const int32_t* c = cord + a;
  const uint8_t* ch = chain + a;
  int32_t ck = 0, cc = -1;
  for (int32_t b = 0; b < M; b += 1024) {
    const int32_t r0 = b + 4 * threadIdx.x;
    int32_t cv[4];
    bool isc[4];
    int2 v = make_int2(0, INT32_MIN);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const bool ok = r0 + q < M;
      cv[q] = ok ? c[r0 + q] : 0;
      isc[q] = ok && ch[r0 + q];
      if (isc[q]) {
        v.x++;
        v.y = cv[q];
      }
    }
    int2 tot;
    const int2 ex = block_scan_cnt_max(v, lds, &tot);
    int32_t kx = ck + ex.x, cx = max(cc, ex.y);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int32_t r = r0 + q;
      if (r < M) {
        if (isc[q]) {
          crow[a + kx] = r;
          kx++;
          cx = cv[q];
        } else {
          posA[a + r] = r + cx + 1 - kx;
        }
      }
    }
    ck += tot.x;
    cc = max(cc, tot.y);
  }
}

// Columns pass: Kc = #chain columns before j; the REMOVE of off-chain column j sits at
// rnext(j) + j - Kc with rnext = row of the Kc-th chain node (M past the last).  Forms both
// entries of every off-chain element x = j (seq = partner position << 2 | type, sx = x) and
// the IGNORE of a chain column j (row r = inv[j], Kr(r) = Kc(j)) at r + j - Kc, right after
// the REMOVEs of its gap: every entry of the sequence comes from this pass.
//
// The entries of a round of columns land within a few dozen positions of one contiguous
// stretch of the sequence (the REMOVE / IGNORE positions ascend with the column, the ADDs of
// the same rows fill the gaps between them), but each one is a single word: stored one by
// one, every store instruction touches a dozen lines and the lines go to memory several times
// over.  So a round collects its entries in an LDS image of the stretch and writes the image
// out with consecutive lanes on consecutive words; slots that no entry of this round fills
// (the ragged ends, which the neighbouring rounds fill) are skipped, and an entry that falls
// outside the image (a far move) is stored directly -- every position is written exactly once
// either way.
__global__ void __launch_bounds__(256) k_pos_cols(const Unit* __restrict__ units, const int32_t* __restrict__ inv,
                                                  const uint8_t* __restrict__ chain, const int32_t* __restrict__ posA,
                                                  const int32_t* __restrict__ crow, uint32_t* __restrict__ seq,
                                                  int32_t* __restrict__ sx) {
  // (rounds of 512 columns: half the LDS of 1024-column rounds, which matters beside the other
  // lanes' kernels, at the same time alone)
  constexpr int32_t PER = 2, ROUND = 256 * PER;
  constexpr int32_t CAP = 2 * ROUND + 256;  // positions of the image (a round makes ~0.8 K entries)
  constexpr int32_t SLACK = 192;  // of them, before the round's first REMOVE / IGNORE position
  constexpr uint32_t kNone = 3u;  // no entry has type 3
  __shared__ int32_t lds[4];
  __shared__ uint32_t wseq[CAP];
  __shared__ int32_t wsx[CAP];
  const Unit u = units[blockIdx.x];
  const int64_t a = u.a;
  const int32_t M = u.M, K = u.K;
  uint32_t* sq = seq + 2 * a;
  int32_t* sxa = sx + 2 * a;
  int32_t ck = 0;
  for (int32_t b = 0; b < M; b += ROUND) {
    const int32_t base = ((ck < K) ? crow[a + ck] : M) + b - ck - SLACK;  // position of image slot 0
    for (int32_t z = threadIdx.x; z < CAP; z += 256) wseq[z] = kNone;
    auto put = [&](int32_t pos, uint32_t e, int32_t x) {
      const int32_t z = pos - base;
      if ((uint32_t)z < (uint32_t)CAP) {
        wseq[z] = e;
        wsx[z] = x;
      } else {
        sq[pos] = e;
        if ((e & 3u) != kIgn) sxa[pos] = x;
      }
    };
    const int32_t j0 = b + PER * threadIdx.x;
    int32_t row[PER];
    bool isc[PER];
    int32_t v = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const bool ok = j0 + q < M;
      row[q] = ok ? inv[a + j0 + q] : 0;
      isc[q] = !ok || chain[a + row[q]];
      v += (ok && isc[q]) ? 1 : 0;
    }
    int32_t tot;
    int32_t kc = ck + block_exclusive_scan<256>(v, 0, OpAdd(), lds, &tot);  // (barriers: the image is cleared)
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const int32_t j = j0 + q;
      if (isc[q]) {
        if (j < M) put(row[q] + j - kc, kIgn, 0);
        kc++;
        continue;
      }
      const int32_t pr = ((kc < K) ? crow[a + kc] : M) + j - kc;
      const int32_t pa = posA[a + row[q]];
      put(pr, ((uint32_t)pa << 2) | kRem, j);
      put(pa, ((uint32_t)pr << 2) | kAdd, j);
    }
    ck += tot;
    __syncthreads();
    for (int32_t z = threadIdx.x; z < CAP; z += 256) {
      const uint32_t e = wseq[z];
      if (e != kNone) {
        sq[base + z] = e;
        if ((e & 3u) != kIgn) sxa[base + z] = wsx[z];
      }
    }
    __syncthreads();
  }
}

// Delta of each off-chain id (convert_to_diff_binary, :358-396), in second-occurrence order
// (the pair order): entries strictly between its two occurrences that are in the decoder's
// list when it moves -- IGNOREs, REMOVEs whose element is still pending (its ADD comes
// later), ADDs whose element has already moved (its REMOVE came earlier).  Negative when the
// second occurrence is the REMOVE.  The pair index is a running count of second occurrences.
//
// One thread per second occurrence walks its span in an LDS ring of the last 2 K sequence
// entries.  The ring holds each entry as one signed word q that makes the test two compares:
// ADD -> partner position (counts when q < s, unsigned), REMOVE -> ~partner (counts when
// q < -s - 1, i.e. partner > s), IGNORE -> INT32_MIN (always counts).  Spans longer than
// kLongSpan are left to whole waves afterwards (64 entries per step), so a trace with far
// moves costs no more than 1/64 of its span per lane.
namespace {
__device__ __forceinline__ int32_t delta_word(uint32_t e) {
  const uint32_t t = e & 3u;
  const int32_t pt = (int32_t)(e >> 2);
  return t == kIgn ? INT32_MIN : (t == kAdd ? pt : ~pt);
}
}  // namespace

__global__ void __launch_bounds__(256, 7) k_deltas(const Unit* __restrict__ units, const uint32_t* __restrict__ seq,
                                                   const int32_t* __restrict__ sx, uint8_t* __restrict__ out) {
  // LDS and registers are kept small (10.3 KB, <= 72 VGPRs): beside the other lanes' kernels the
  // LDS left on a CU decides how many blocks run.  Rounds of ROUND sequence entries, PER per thread.
  constexpr int32_t PER = 2, ROUND = 256 * PER;
  constexpr int32_t RING = 2 * ROUND;  // the last RING sequence entries, for the span counts
  constexpr int32_t kLongSpan = 192;
  static_assert(RING - ROUND > kLongSpan, "a short span must lie in the ring");
  __shared__ int32_t lds[4];
  __shared__ int2 items[ROUND];  // second occurrences of the round: {position s, entry}, then {s, delta}
  __shared__ int32_t ring[RING];
  __shared__ int32_t longs[ROUND];  // items of the round with long spans; then the ids of the round's pairs
  __shared__ int32_t nlong;
  __shared__ int32_t carry[4];     // the last two ids and the last two deltas before this round (LP)
  const Unit u = units[blockIdx.x];
  const int64_t a = u.a;
  const uint32_t* sq = seq + 2 * a;
  const int32_t L = 2 * u.P + u.K;
  const int32_t* sxa = sx + 2 * a;
  int32_t ck = 0;
  // The pairs go straight into the unit's pair section of the file, linear-predicted
  // (compress_matched_events :706-721; x[i] - 2 x[i-1] + x[i-2] in 32 bits,
  // rempi_compression_util.cpp:117-154): ids at the section start, deltas P words later.
  uint8_t* const osec = out + u.out_off + 72 + 16ll * u.S + 8ll * u.W + 8ll * u.M + 16ll * u.U;
  if (threadIdx.x < 4) carry[threadIdx.x] = 0;
  // this round's sequence entries; the next round's are loaded while the spans of this one
  // are counted
  uint32_t e[PER];
#pragma unroll
  for (int q = 0; q < PER; q++) {
    const int32_t z = PER * threadIdx.x + q;
    e[q] = (z < L) ? sq[z] : kIgn;
  }
  for (int32_t b = 0; b < L; b += ROUND) {
    const int32_t q0 = b + PER * threadIdx.x;
    int32_t v = 0;
#pragma unroll
    for (int q = 0; q < PER; q++)
      if ((e[q] & 3) != kIgn && (int32_t)(e[q] >> 2) < q0 + q) v++;
    int32_t tot;
    int32_t k = block_exclusive_scan<256>(v, 0, OpAdd(), lds, &tot);
    if (threadIdx.x == 0) nlong = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) {
      ring[(q0 + q) & (RING - 1)] = delta_word(e[q]);
      if ((e[q] & 3) != kIgn && (int32_t)(e[q] >> 2) < q0 + q) items[k++] = make_int2(q0 + q, (int32_t)e[q]);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const int32_t z = q0 + ROUND + q;
      e[q] = (z < L) ? sq[z] : kIgn;
    }
    const int32_t rlo = b + ROUND - RING;  // entries >= rlo are in the ring
    for (int32_t it = threadIdx.x; it < tot; it += 256) {
      const int2 item = items[it];
      const int32_t s = item.x, f = (int32_t)((uint32_t)item.y >> 2);
      if (s - f - 1 > kLongSpan || f + 1 < rlo) {
        longs[atomicAdd(&nlong, 1)] = it;
        continue;
      }
      const int32_t ns1 = -s - 1;
      int32_t d = 0;
      for (int32_t z = f + 1; z < s; z++) {
        const int32_t q = ring[z & (RING - 1)];
        d += ((uint32_t)q < (uint32_t)s || q < ns1) ? 1 : 0;
      }
      items[it].y = (((uint32_t)item.y & 3) == kRem) ? -d : d;
    }
    __syncthreads();
    // long spans, and spans that reach behind the ring (entries more than half a ring back come from
    // memory): one wave per item
    for (int32_t li = wave_id(); li < nlong; li += 4) {
      const int32_t it = longs[li];
      const int2 item = items[it];
      const int32_t s = item.x, f = (int32_t)((uint32_t)item.y >> 2);
      const int32_t ns1 = -s - 1;
      int32_t d = 0;
      for (int32_t z0 = f + 1; z0 < s; z0 += 64) {
        const int32_t z = z0 + lane_id();
        bool c = false;
        if (z < s) {
          const int32_t q = z >= rlo ? ring[z & (RING - 1)] : delta_word(sq[z]);
          c = (uint32_t)q < (uint32_t)s || q < ns1;
        }
        d += __popcll(__builtin_amdgcn_ballot_w64(c));
      }
      if (lane_id() == 0) items[it].y = (((uint32_t)item.y & 3) == kRem) ? -d : d;
    }
    __syncthreads();
    for (int32_t q = threadIdx.x; q < tot; q += 256) longs[q] = sxa[items[q].x];  // the pairs' ids
    __syncthreads();
    for (int32_t q = threadIdx.x; q < tot; q += 256) {  // the round's pairs, coalesced
      const uint32_t i0 = (uint32_t)longs[q], d0 = (uint32_t)items[q].y;
      const uint32_t i1 = q >= 1 ? (uint32_t)longs[q - 1] : (uint32_t)carry[0];
      const uint32_t d1 = q >= 1 ? (uint32_t)items[q - 1].y : (uint32_t)carry[2];
      const uint32_t i2 = q >= 2 ? (uint32_t)longs[q - 2] : (uint32_t)carry[1 - q];
      const uint32_t d2 = q >= 2 ? (uint32_t)items[q - 2].y : (uint32_t)carry[3 - q];
      st_u32(osec + 4ll * (ck + q), i0 - 2 * i1 + i2);
      st_u32(osec + 4ll * u.P + 4ll * (ck + q), d0 - 2 * d1 + d2);
    }
    __syncthreads();
    if (threadIdx.x == 0 && tot > 0) {
      const int32_t pi = carry[0], pd = carry[2];
      carry[1] = tot >= 2 ? longs[tot - 2] : pi;
      carry[3] = tot >= 2 ? items[tot - 2].y : pd;
      carry[0] = longs[tot - 1];
      carry[2] = items[tot - 1].y;
    }
    ck += tot;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// Serialization of one unit (compress_non_matched_events :627-703,
// compress_matched_events :706-721, LP of rempi_compression_util.cpp:117-154).
__device__ __forceinline__ uint64_t lp64(const int32_t* x, int32_t i) {
  const uint64_t v0 = sext(x[i]);
  const uint64_t v1 = i >= 1 ? sext(x[i - 1]) : 0;
  const uint64_t v2 = i >= 2 ? sext(x[i - 2]) : 0;
  return v0 - 2 * v1 + v2;
}

__global__ void __launch_bounds__(256) k_write_units(const Unit* __restrict__ units, const int32_t* __restrict__ midx,
                                                     const int32_t* __restrict__ wp, const int32_t* __restrict__ run_id,
                                                     const uint64_t* __restrict__ run_cnt,
                                                     const uint64_t* __restrict__ ep_rank,
                                                     const uint64_t* __restrict__ ep_clk, int64_t ep_stride, int32_t rep,
                                                     uint8_t* __restrict__ out) {
  Unit u = units[blockIdx.x];
  const int64_t a = u.a;
  const int64_t ea = epoch_slot(blockIdx.x, a, ep_stride);
  uint8_t* o = out + u.out_off;
  const int t = threadIdx.x;
  // REMPI_ENCODE=7 (rempi_encoder_rep.cpp:50-146): the same table with every section after
  // the epoch line empty (lengths and sizes 0); the count stays the matched-event count.
  const int32_t count = u.M;
  if (rep) u.W = u.M = u.U = u.P = 0;
  if (t == 0) {
    st_u32(o, (uint32_t)u.set_id);
    st_u32(o + 4, (uint32_t)count);
    st_u64(o + 8, 8ull * u.S);
  }
  uint8_t* p = o + 16;
  for (int i = t; i < u.S; i += 256) {
    st_u64(p + 8 * i, ep_rank[ea + i]);
    st_u64(p + 8 * (u.S + i), ep_clk[ea + i]);
  }
  p += 16ull * u.S;
  if (t == 0) {
    st_u64(p, (uint64_t)u.W);
    st_u64(p + 8, 8ull * u.W);
  }
  p += 16;
  for (int i = t; i < u.W; i += 256) st_u64(p + 8 * i, lp64(wp + a, i));
  p += 8ull * u.W;
  if (t == 0) {
    st_u64(p, (uint64_t)u.M);
    st_u64(p + 8, 8ull * u.M);
  }
  p += 16;
  for (int i = t; i < u.M; i += 256) st_u64(p + 8 * i, sext(midx[a + i]));
  p += 8ull * u.M;
  if (t == 0) st_u64(p, 8ull * u.U);
  p += 8;
  for (int i = t; i < u.U; i += 256) st_u64(p + 8 * i, lp64(run_id + a, i));
  p += 8ull * u.U;
  if (t == 0) st_u64(p, 8ull * u.U);
  p += 8;
  for (int i = t; i < u.U; i += 256) st_u64(p + 8 * i, run_cnt[a + i]);
  p += 8ull * u.U;
  if (t == 0) st_u64(p, 8ull * u.P);  // (the pairs themselves: k_deltas)
}

__global__ void __launch_bounds__(256) k_chunk_headers(const Chunk* __restrict__ ch, int32_t n, uint8_t* __restrict__ out) {
  latency_kernel();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) st_u64(out + ch[i].out_off, (uint64_t)ch[i].payload);
}

// Footer (write_footer, :2085-2126): all_epoch_rank_uset (unordered_set<int>) fed with
// every table's epoch ranks in emitted order.  Its iteration order depends only on the
// distinct keys in first-insertion order, so one block per rank first finds each distinct
// key's first position (LDS hash, atomicMin of (unit, slot)), sorts the distinct keys by it,
// and only then replays the libstdc++ insertions -- one per distinct key instead of one
// membership walk per (table, source).  A rank with more distinct keys than the LDS hash
// holds replays every insertion sequentially.
__global__ void __launch_bounds__(256) k_footer_order(const Unit* __restrict__ units, const int32_t* __restrict__ ufirst,
                                                      const int32_t* __restrict__ nunits, const uint64_t* __restrict__ ep_rank,
                                                      int64_t ep_stride, int32_t n_ranks, const int64_t* __restrict__ fk_off,
                                                      const int64_t* __restrict__ fb_off, uint64_t* __restrict__ fkey,
                                                      int32_t* __restrict__ fnext, int32_t* __restrict__ fbucket,
                                                      int32_t* __restrict__ fcount) {
  latency_kernel();
  constexpr int HC = 4096, LCAP = HC / 2;
  __shared__ int32_t hkey[HC];
  __shared__ unsigned long long hord[HC];
  __shared__ int32_t nlist;
  const int r = blockIdx.x;
  if (r >= n_ranks) return;
  for (int i = threadIdx.x; i < HC; i += 256) {
    hkey[i] = INT32_MIN;
    hord[i] = ~0ull;
  }
  if (threadIdx.x == 0) nlist = 0;
  __syncthreads();
  const int32_t nu = nunits[r], u0 = ufirst[r];
  const int w = wave_id(), l = lane_id();
  for (int32_t q = w; q < nu; q += 4) {
    const Unit u = units[u0 + q];
    for (int32_t j = l; j < u.S; j += 64) {
      const int32_t k = (int32_t)ep_rank[epoch_slot(u0 + q, u.a, ep_stride) + j];
      const unsigned long long ord = ((unsigned long long)q << 12) | (unsigned long long)j;
      uint32_t h = ((uint32_t)k * 2654435761u) % HC;
      for (int probe = 0; probe < HC; probe++) {
        const int32_t old = atomicCAS(&hkey[h], INT32_MIN, k);
        if (old == INT32_MIN) atomicAdd(&nlist, 1);
        if (old == INT32_MIN || old == k) {
          atomicMin(&hord[h], ord);
          break;
        }
        h = (h + 1) % HC;
      }
    }
  }
  __syncthreads();
  const int n = nlist;
  HashOrder ho;
  if (n > LCAP) {  // too many distinct keys for the LDS list: sequential replay
    if (threadIdx.x == 0) {
      ho.init(fkey + fk_off[r], fnext + fk_off[r], fbucket + fb_off[r]);
      for (int32_t q = 0; q < nu; q++) {
        const Unit u = units[u0 + q];
        for (int32_t j = 0; j < u.S; j++) {
          const uint64_t k = (uint64_t)(int64_t)(int32_t)ep_rank[epoch_slot(u0 + q, u.a, ep_stride) + j];
          if (!ho.contains(k)) ho.insert_new(k);
        }
      }
      fcount[r] = ho.size;
      fbucket[fb_off[r]] = ho.head;
    }
    return;
  }
  // Compact the table into the front of its own storage (every thread first takes its share of
  // the slots into registers), then bitonic sort by order.
  int32_t* const lkey = hkey;
  unsigned long long* const lord = hord;
  __shared__ int32_t cnt;
  int32_t ck[HC / 256];
  unsigned long long co[HC / 256];
#pragma unroll
  for (int q = 0; q < HC / 256; q++) {
    ck[q] = hkey[q * 256 + threadIdx.x];
    co[q] = hord[q * 256 + threadIdx.x];
  }
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < HC / 256; q++) {
    if (ck[q] != INT32_MIN) {
      const int at = atomicAdd(&cnt, 1);
      lkey[at] = ck[q];
      lord[at] = co[q];
    }
  }
  int P2 = 1;
  while (P2 < n) P2 <<= 1;
  __syncthreads();
  for (int i = n + threadIdx.x; i < P2; i += 256) lord[i] = ~0ull;
  __syncthreads();
  for (int size = 2; size <= P2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int p = threadIdx.x; p < P2 / 2; p += 256) {
        const int i = 2 * p - (p & (stride - 1));
        const int j = i + stride;
        const bool up = ((i & size) == 0);
        if ((lord[i] > lord[j]) == up) {
          const unsigned long long t = lord[i];
          lord[i] = lord[j];
          lord[j] = t;
          const int32_t tk = lkey[i];
          lkey[i] = lkey[j];
          lkey[j] = tk;
        }
      }
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) {
    ho.init(fkey + fk_off[r], fnext + fk_off[r], fbucket + fb_off[r]);
    for (int q = 0; q < n; q++) ho.insert_new((uint64_t)(int64_t)lkey[q]);
    fcount[r] = ho.size;
    fbucket[fb_off[r]] = ho.head;
  }
}

__global__ void __launch_bounds__(64) k_footer_write(const int64_t* __restrict__ fk_off, const int64_t* __restrict__ fb_off,
                                                     const uint64_t* __restrict__ fkey, const int32_t* __restrict__ fnext,
                                                     const int32_t* __restrict__ fbucket, const int32_t* __restrict__ fcount,
                                                     const int64_t* __restrict__ foot_off, int32_t n_ranks,
                                                     uint8_t* __restrict__ out) {
  latency_kernel();
  const int r = blockIdx.x * 64 + threadIdx.x;
  if (r >= n_ranks) return;
  uint8_t* o = out + foot_off[r];
  st_u64(o, 0);
  st_u64(o + 8, (uint64_t)fcount[r]);
  int32_t j = 0;
  const int64_t kb = fk_off[r];
  for (int32_t p = fbucket[fb_off[r]]; p != -1; p = fnext[kb + p], j++) st_u32(o + 16 + 4 * j, (uint32_t)fkey[kb + p]);
  st_u32(o + 16 + 4ull * fcount[r], 0);
}

}  // namespace cdcx
