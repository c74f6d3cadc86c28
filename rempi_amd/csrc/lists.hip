// lists.hip -- the work lists of a batch, built on the device.
//
// The record side needs, in this order: the record tiles, the chunk list (after k_chunks), the
// (chunk, table) units (after k_units_lb), the sort tiles and key offsets (after k_unit_prep),
// the segment offsets (after k_cuts) and the output layout (after k_deltas and k_footer_order).
// The replay side needs the unit offsets, the launch order of the permutation rebuild and the
// record tiles.  Every one of them is a scan over a few thousand descriptors: a single
// workgroup does it in a few dozen rounds, and the host only reads back the handful
// of totals that size buffers and grids (EncTotals / DecTotals) instead of downloading,
// walking and re-uploading the descriptor arrays between kernels.  (256 threads, not 1024: a
// workgroup needs all its wave slots on one CU, and while other streams' kernels fill the CUs
// a 16-wave workgroup waited milliseconds for a CU with room -- the scans took 1.2-3.4 ms each
// under load against 0.07 ms alone.)
#include <hip/hip_runtime.h>

#include "cdcx_device.h"
#include "cdcx_kernels.h"

namespace cdcx {

namespace {

// Exclusive scan of v over the block's threads plus a running carry; returns the exclusive
// prefix including the carry and advances the carry by the round's total.
template <class T>
__device__ __forceinline__ T scan_round(T v, T& carry, T* lds) {
  T tot;
  const T ex = block_exclusive_scan<kScanBlock>(v, T(0), OpAdd(), lds, &tot);
  const T r = carry + ex;
  carry += tot;
  return r;
}
}  // namespace

// Record tiles of every rank: tile q of rank r covers records [q * kTile, ...) of the rank.
__global__ void __launch_bounds__(256) k_build_tiles(const int64_t* __restrict__ rec_off, const int32_t* __restrict__ tile0,
                                                     Tile* __restrict__ tiles) {
  latency_kernel();
  const int r = blockIdx.x;
  const int64_t b = rec_off[r], n = rec_off[r + 1] - b;
  for (int64_t q = threadIdx.x; q * kTile < n; q += 256)
    tiles[tile0[r] + q] = Tile{r, (int32_t)min((int64_t)kTile, n - q * kTile), b + q * kTile, (int32_t)q, 0};
}

// Chunk descriptors in (rank, chunk) order from the per-rank boundary lists of k_chunks.
// cbase[r] = chunks of earlier ranks, lbase[r] = (chunk, table) slots of earlier ranks.
__global__ void __launch_bounds__(256) k_build_chunks(const int2* __restrict__ chunk_cap, const int64_t* __restrict__ ccap_off,
                                                      const int32_t* __restrict__ nchunks, const int32_t* __restrict__ nsets,
                                                      const int32_t* __restrict__ cbase, const int64_t* __restrict__ lbase,
                                                      Chunk* __restrict__ chunks, int64_t* __restrict__ lb_off) {
  latency_kernel();
  const int r = blockIdx.x;
  const int32_t n = nchunks[r], T = nsets[r];
  for (int32_t k = threadIdx.x; k < n; k += 256) {
    const int2 se = chunk_cap[ccap_off[r] + k];
    chunks[cbase[r] + k] = Chunk{r, se.x, se.y, 0, 0, 0, 0, 0};
    lb_off[cbase[r] + k] = lbase[r] + (int64_t)k * T;
  }
}

// First unit of every chunk and of every rank, the chunks' offsets into the lane-tier leaf
// scratch (one row per record of a unit plus one), the unit count.  ucnt / uw: non-empty
// tables and sum of (records + 1) of each chunk (k_units_lb).
__global__ void __launch_bounds__(kScanBlock) k_scan_chunks(Chunk* __restrict__ chunks, int32_t C,
                                                            const int32_t* __restrict__ ucnt, const int64_t* __restrict__ uw,
                                                            const int32_t* __restrict__ cbase, int32_t R,
                                                            int32_t* __restrict__ ufirst, int32_t* __restrict__ nunits,
                                                            int64_t* __restrict__ cw1, EncTotals* __restrict__ tot) {
  latency_kernel();
  __shared__ int64_t lds[kScanBlock / kWave];
  int64_t cu = 0, cw = 0;
  for (int32_t b = 0; b < C; b += kScanBlock) {
    const int32_t c = b + threadIdx.x;
    const int64_t n = c < C ? ucnt[c] : 0, w = c < C ? uw[c] : 0;
    const int64_t fu = scan_round(n, cu, lds), fw = scan_round(w, cw, lds);
    if (c < C) {
      chunks[c].first_unit = (int32_t)fu;
      chunks[c].n_units = (int32_t)n;
      cw1[c] = fw;
    }
  }
  __syncthreads();
  for (int32_t r = threadIdx.x; r < R; r += kScanBlock) {
    const int32_t c0 = cbase[r], c1 = cbase[r + 1];
    const int32_t f0 = c0 < C ? chunks[c0].first_unit : (int32_t)cu, f1 = c1 < C ? chunks[c1].first_unit : (int32_t)cu;
    ufirst[r] = f0;
    nunits[r] = f1 - f0;
  }
  if (threadIdx.x == 0) {
    tot->n_units = (int32_t)cu;
    tot->w1n = cw;
  }
}

// The units of one chunk: its non-empty tables in ascending set id (lohi from k_units_lb).
__global__ void __launch_bounds__(kMaxSets) k_fill_units(const Chunk* __restrict__ chunks, const int64_t* __restrict__ lb_off,
                                                         const int2* __restrict__ lohi, const int32_t* __restrict__ nsets,
                                                         const int32_t* __restrict__ setlist,
                                                         const int64_t* __restrict__ rec_off, const int64_t* __restrict__ cw1,
                                                         Unit* __restrict__ units, int64_t* __restrict__ w1) {
  latency_kernel();
  __shared__ int64_t lds[kMaxSets / kWave];
  const int32_t c = blockIdx.x;
  const Chunk C = chunks[c];
  const int tb = threadIdx.x;
  int2 lh = make_int2(0, 0);
  if (tb < nsets[C.rank]) lh = lohi[lb_off[c] + tb];
  const bool has = lh.y > lh.x;
  const int64_t n = has ? lh.y - lh.x : 0;
  // one scan for both prefixes: the unit count in the high bits, the rows below
  int64_t tot;
  const int64_t ex = block_exclusive_scan<kMaxSets>(has ? ((int64_t)1 << 40) + n + 1 : 0, (int64_t)0, OpAdd(), lds, &tot);
  if (has) {
    const int32_t ui = C.first_unit + (int32_t)(ex >> 40);
    Unit u{};
    u.a = rec_off[C.rank] + lh.x;
    u.n = (int32_t)n;
    u.rank = C.rank;
    u.chunk = c;
    u.set_id = setlist[(size_t)C.rank * kMaxSets + tb];
    units[ui] = u;
    w1[ui] = cw1[c] + (ex & (((int64_t)1 << 40) - 1));
  }
}

// After k_unit_prep: first sort tile and sorted-key offset of every unit, the windowed-rank
// flag (1 = take the tile sort), totals.
__global__ void __launch_bounds__(kScanBlock) k_units_scan_prep(Unit* __restrict__ units, int32_t rank_tier,
                                                                EncTotals* __restrict__ tot) {
  latency_kernel();
  __shared__ int64_t lds[kScanBlock / kWave];
  const int32_t NU = tot->n_units;
  int64_t ct = 0, cm = 0, cw = 0, cr = 0;
  for (int32_t b = 0; b < NU; b += kScanBlock) {
    const int32_t u = b + threadIdx.x;
    const bool ok = u < NU;
    const int64_t M = ok ? units[u].M : 0;
    const int64_t t0 = scan_round((M + kSortTile - 1) / kSortTile, ct, lds);
    const int64_t k0 = scan_round(M, cm, lds);
    (void)scan_round(ok ? (int64_t)units[u].W : 0, cw, lds);
    (void)scan_round(ok ? (int64_t)units[u].U : 0, cr, lds);
    if (ok) {
      units[u].sort_tile0 = (int32_t)t0;
      units[u].key_off = k0;
      units[u].wfail = rank_tier > 0 ? 1 : 0;
    }
  }
  if (threadIdx.x == 0) {
    tot->n_sort_tiles = (int32_t)ct;
    tot->matched = cm;
    tot->with_next = cw;
    tot->runs = cr;
  }
}

__global__ void __launch_bounds__(256) k_fill_sort_tiles(const Unit* __restrict__ units, SortTile* __restrict__ st) {
  latency_kernel();
  const Unit u = units[blockIdx.x];
  for (int32_t q = threadIdx.x; q * kSortTile < u.M; q += 256) st[u.sort_tile0 + q] = SortTile{(int32_t)blockIdx.x, q};
}

// After k_epoch and k_cuts: first segment of every unit, the units the windowed rank failed on
// and those with more sources than the small epoch instance holds, epoch sources per rank
// (bound[], zeroed by the host) and in total.
__global__ void __launch_bounds__(kScanBlock) k_units_scan_cuts(Unit* __restrict__ units, int64_t* __restrict__ bound,
                                                                EncTotals* __restrict__ tot) {
  latency_kernel();
  __shared__ int64_t lds[kScanBlock / kWave];
  const int32_t NU = tot->n_units;
  int64_t cs = 0, cf = 0, cb = 0, ce = 0;
  for (int32_t b = 0; b < NU; b += kScanBlock) {
    const int32_t u = b + threadIdx.x;
    const bool ok = u < NU;
    const int32_t S = ok ? units[u].S : 0;
    const int64_t s0 = scan_round(ok ? (int64_t)units[u].nseg : 0, cs, lds);
    (void)scan_round((int64_t)(ok && units[u].wfail == 1), cf, lds);
    (void)scan_round((int64_t)(ok && S == -1), cb, lds);
    (void)scan_round((int64_t)max(S, 0), ce, lds);
    if (ok) {
      units[u].seg0 = (int32_t)min(s0, (int64_t)INT32_MAX);
      if (S > 0) atomicAdd(reinterpret_cast<unsigned long long*>(&bound[units[u].rank]), (unsigned long long)S);
    }
  }
  if (threadIdx.x == 0) {
    tot->n_segs = cs;
    tot->n_fail = (int32_t)cf;
    tot->n_big = (int32_t)cb;
    tot->sources = ce;
  }
}

__global__ void __launch_bounds__(256) k_units_clear_wfail(Unit* __restrict__ units, int32_t NU) {
  latency_kernel();
  const int32_t u = blockIdx.x * 256 + threadIdx.x;
  if (u < NU) units[u].wfail = 0;
}

// Output layout (write_record_file framing): every rank file starts 16-byte aligned and holds
// its chunks ([size_t payload][tables]...) and the footer (20 + 4 * distinct epoch ranks).
// Fills Unit::out_off, Chunk::out_off / payload, the files' offsets and lengths, the footers'
// offsets and the batch total.  upre / cpre: scratch of n_units + 1 / C + 1 words.
__global__ void __launch_bounds__(kScanBlock) k_out_layout(Unit* __restrict__ units, Chunk* __restrict__ chunks, int32_t C,
                                                           const int32_t* __restrict__ cbase, int32_t R,
                                                           const int32_t* __restrict__ fcount, int32_t rep,
                                                           const EncTotals* __restrict__ tot, int64_t* __restrict__ upre,
                                                           int64_t* __restrict__ cpre, int64_t* __restrict__ file_off,
                                                           int64_t* __restrict__ file_len, int64_t* __restrict__ foot_off,
                                                           int64_t* __restrict__ total) {
  latency_kernel();
  __shared__ int64_t lds[kScanBlock / kWave];
  const int32_t NU = tot->n_units;
  int64_t carry = 0;
  for (int32_t b = 0; b < NU; b += kScanBlock) {
    const int32_t q = b + threadIdx.x;
    int64_t sz = 0;
    if (q < NU) {
      const Unit& u = units[q];
      sz = 72 + 16ll * u.S + (rep ? 0 : 8ll * u.W + 8ll * u.M + 16ll * u.U + 8ll * u.P);
    }
    const int64_t ex = scan_round(sz, carry, lds);
    if (q < NU) upre[q] = ex;
  }
  if (threadIdx.x == 0) upre[NU] = carry;
  __syncthreads();
  carry = 0;
  for (int32_t b = 0; b < C; b += kScanBlock) {
    const int32_t c = b + threadIdx.x;
    int64_t sz = 0;
    if (c < C) sz = 8 + upre[chunks[c].first_unit + chunks[c].n_units] - upre[chunks[c].first_unit];
    const int64_t ex = scan_round(sz, carry, lds);
    if (c < C) cpre[c] = ex;
  }
  if (threadIdx.x == 0) cpre[C] = carry;
  __syncthreads();
  carry = 0;
  for (int32_t b = 0; b < R; b += kScanBlock) {
    const int32_t r = b + threadIdx.x;
    int64_t fsz = 0;
    if (r < R) fsz = cpre[cbase[r + 1]] - cpre[cbase[r]] + 20 + 4ll * fcount[r];
    const int64_t ex = scan_round((fsz + 15) / 16 * 16, carry, lds);
    if (r < R) {
      file_off[r] = ex;
      file_len[r] = fsz;
      foot_off[r] = ex + fsz - (20 + 4ll * fcount[r]);
    }
  }
  if (threadIdx.x == 0) {
    total[0] = carry;
    total[1] = upre[NU];  // bytes of all tables (the host reads the number of pairs off it)
  }
  __syncthreads();
  for (int32_t c = threadIdx.x; c < C; c += kScanBlock) {
    Chunk& ch = chunks[c];
    ch.out_off = file_off[ch.rank] + cpre[c] - cpre[cbase[ch.rank]];
    ch.payload = upre[ch.first_unit + ch.n_units] - upre[ch.first_unit];
  }
  __syncthreads();
  for (int32_t q = threadIdx.x; q < NU; q += kScanBlock) {
    Unit& u = units[q];
    const Chunk& ch = chunks[u.chunk];
    u.out_off = ch.out_off + 8 + upre[q] - upre[ch.first_unit];
  }
}

// ---------------------------------------------------------------------------------------
// Replay side.

// First unit of every chunk from the per-chunk unit counts of k_dec_units' counting pass.
__global__ void __launch_bounds__(kScanBlock) k_dec_scan_chunks(const int32_t* __restrict__ nu, int32_t C,
                                                                int32_t* __restrict__ first_unit, DecTotals* __restrict__ tot) {
  latency_kernel();
  __shared__ int64_t lds[kScanBlock / kWave];
  int64_t carry = 0;
  for (int32_t b = 0; b < C; b += kScanBlock) {
    const int32_t c = b + threadIdx.x;
    const int64_t ex = scan_round(c < C ? (int64_t)nu[c] : 0, carry, lds);
    if (c < C) first_unit[c] = (int32_t)min(ex, (int64_t)INT32_MAX);
  }
  if (threadIdx.x == 0) tot->n_units = carry;
}

// Scratch, record and key offsets of every unit (file order), its first record tile, the first
// permutation-rebuild tier, totals.
__global__ void __launch_bounds__(kScanBlock) k_dec_scan_units(DUnit* __restrict__ units, int32_t NU, int32_t tier,
                                                               int32_t* __restrict__ tile0, DecTotals* __restrict__ tot) {
  latency_kernel();
  __shared__ int64_t lds[kScanBlock / kWave];
  int64_t cw = 0, cr = 0, ck = 0, ct = 0, cs = 0;
  for (int32_t b = 0; b < NU; b += kScanBlock) {
    const int32_t q = b + threadIdx.x;
    const bool ok = q < NU;
    int64_t M = 0, nrun = 0;
    int32_t nseg = 0;
    if (ok) {
      M = units[q].M;
      nrun = units[q].Uc > 0 ? units[q].U : 0;
      nseg = dec_nseg(units[q].P);
    }
    const int64_t w0 = scan_round(ok ? M + 1 : 0, cw, lds);
    const int64_t r0 = scan_round(M + nrun, cr, lds);
    const int64_t k0 = scan_round(M, ck, lds);
    const int64_t t0 = scan_round((int64_t)((ok && (M > 0 || nrun > 0)) ? max((M + kRecTile - 1) / kRecTile, (int64_t)1) : 0), ct, lds);
    const int64_t s0 = scan_round((int64_t)nseg, cs, lds);
    if (ok) {
      units[q].nseg = nseg;
      units[q].seg0 = s0;
      units[q].wbase = w0;
      units[q].rec_off = r0;
      units[q].key_off = k0;
      units[q].fb = tier;
      tile0[q] = (int32_t)t0;
    }
  }
  if (threadIdx.x == 0) {
    if (NU > 0) tile0[NU] = (int32_t)ct;
    tot->rows = cw;
    tot->records = cr;
    tot->keys = ck;
    tot->rec_tiles = ct;
    tot->segs = cs;
  }
}

// Launch order of the permutation rebuild: units by descending pair count, equal counts in file
// order (a stable sort by counting: order[#units that come before q] = q).
__global__ void __launch_bounds__(256) k_dec_order(const DUnit* __restrict__ units, int32_t NU, int32_t* __restrict__ order) {
  latency_kernel();
  __shared__ int32_t tp[256];
  const int32_t q = blockIdx.x * 256 + threadIdx.x;
  const int32_t P = q < NU ? units[q].P : 0;
  int32_t before = 0;
  for (int32_t b = 0; b < NU; b += 256) {
    __syncthreads();
    tp[threadIdx.x] = (b + threadIdx.x < NU) ? units[b + threadIdx.x].P : -1;
    __syncthreads();
    const int32_t n = min(256, NU - b);
    for (int32_t k = 0; k < n; k++) before += (tp[k] > P || (tp[k] == P && b + k < q)) ? 1 : 0;
  }
  if (q < NU) order[before] = q;
}

// Record tiles of k_dec_records: {unit, tile} for every 1024 matched rows of a unit (at least
// one tile for a unit that only holds unmatched runs).
__global__ void __launch_bounds__(256) k_dec_fill_tiles(const DUnit* __restrict__ units, const int32_t* __restrict__ tile0,
                                                        const uint64_t* __restrict__ uidd, int4* __restrict__ tiles) {
  latency_kernel();
  const int32_t q = blockIdx.x;
  const DUnit u = units[q];
  const int32_t t0 = tile0[q], n = tile0[q + 1] - t0;
  const int32_t U = (u.Uc > 0) ? u.U : 0;
  const uint64_t* ids = uidd + u.wbase;
  // the unmatched runs that precede the tile's rows (ids ascending; a run with id == M follows the last row)
  auto lower = [&](uint64_t key) {
    int32_t lo = 0, hi = U;
    while (lo < hi) {
      const int32_t mid = (lo + hi) >> 1;
      if (ids[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
  };
  for (int32_t k = threadIdx.x; k < n; k += 256) {
    const int64_t i0 = (int64_t)k * kRecTile;
    const bool last = i0 + kRecTile >= u.M;
    tiles[t0 + k] = make_int4(q, k, lower((uint64_t)i0), lower(last ? (uint64_t)u.M + 1 : (uint64_t)(i0 + kRecTile)));
  }
}

}  // namespace cdcx
