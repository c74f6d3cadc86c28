// decode.hip -- CDC replay-side kernels for gfx950.
//
//   framing walk (read_record_file :933-978) -> unit section table (decode :1044-1200)
//   -> inverse linear prediction of with_previous / unmatched ids / ids / delays as two
//   chained prefix sums (rempi_compression_util.cpp:157-168) -> permutation rebuild
//   (cdc_prepare_decode_indices :1301-1386) -> per-table observed record stream.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "cdcx_device.h"
#include "cdcx_kernels.h"

namespace cdcx {

// One lane per rank file: count chunks, validate the framing and the footer.
__global__ void __launch_bounds__(64) k_dec_count_chunks(const uint8_t* __restrict__ in, const int64_t* __restrict__ off,
                                                         const int64_t* __restrict__ len, int32_t n_ranks,
                                                         int32_t* __restrict__ nchunks, uint32_t* err) {
  latency_kernel();
  const int r = blockIdx.x * 64 + threadIdx.x;
  if (r >= n_ranks) return;
  const uint8_t* b = in + off[r];
  const int64_t L = len[r];
  int64_t p = 0;
  int32_t k = 0;
  while (true) {
    if (p + 8 > L) { raise_error(err, kErrCorrupt); break; }
    const uint64_t n = ld_u64(b + p);
    p += 8;
    if (n == 0) {
      if (p + 8 > L) { raise_error(err, kErrCorrupt); break; }
      const uint64_t nr = ld_u64(b + p);
      if (nr > (uint64_t)L || p + 8 + 4 * (int64_t)nr + 4 > L) raise_error(err, kErrCorrupt);
      break;
    }
    if ((n & 7) || n > (uint64_t)(L - p)) { raise_error(err, kErrCorrupt); break; }
    p += (int64_t)n;
    k++;
  }
  nchunks[r] = k;
}

__global__ void __launch_bounds__(64) k_dec_list_chunks(const uint8_t* __restrict__ in, const int64_t* __restrict__ off,
                                                        const int32_t* __restrict__ cbase, const int32_t* __restrict__ nchunks,
                                                        int32_t n_ranks, DChunk* __restrict__ chunks) {
  latency_kernel();
  const int r = blockIdx.x * 64 + threadIdx.x;
  if (r >= n_ranks) return;
  int64_t p = off[r];
  for (int32_t k = 0; k < nchunks[r]; k++) {
    const uint64_t n = ld_u64(in + p);
    chunks[cbase[r] + k] = DChunk{p + 8, (int64_t)n, r, 0};
    p += 8 + (int64_t)n;
  }
}

// Walk the tables of one chunk payload.  When `units` is null only counts.
__device__ bool walk_units(const uint8_t* __restrict__ in, const DChunk& c, int32_t first_unit, DUnit* units,
                           int32_t* count, int32_t max_units = INT32_MAX) {
  int64_t q = c.off;
  const int64_t end = c.off + c.len;
  int32_t k = 0;
  auto need = [&](int64_t bytes) { return q + bytes <= end; };
  while (q < end) {
    DUnit u{};
    u.base = q;
    u.rank = c.rank;
    if (!need(16)) return false;
    u.set_id = (int32_t)ld_u32(in + q);
    u.M = (int32_t)ld_u32(in + q + 4);
    const uint64_t esz = ld_u64(in + q + 8);
    if ((esz & 7) || esz > (uint64_t)(end - q)) return false;
    u.S = (int32_t)(esz / 8);
    u.ep_off = q + 16;
    q += 16 + 2 * (int64_t)esz;
    if (!need(16)) return false;
    const uint64_t wsz = ld_u64(in + q + 8);
    if ((wsz & 7) || wsz > (uint64_t)(end - q)) return false;
    u.W = (int32_t)(wsz / 8);
    u.wp_off = q + 16;
    q += 16 + (int64_t)wsz;
    if (!need(16)) return false;
    const uint64_t msz = ld_u64(in + q + 8);
    if ((msz & 7) || msz > (uint64_t)(end - q)) return false;
    u.Mi = (int32_t)(msz / 8);
    u.mi_off = q + 16;
    q += 16 + (int64_t)msz;
    if (!need(8)) return false;
    const uint64_t usz = ld_u64(in + q);
    if ((usz & 7) || usz > (uint64_t)(end - q)) return false;
    u.U = (int32_t)(usz / 8);
    u.uid_off = q + 8;
    q += 8 + (int64_t)usz;
    if (!need(8)) return false;
    const uint64_t csz = ld_u64(in + q);
    if ((csz & 7) || csz > (uint64_t)(end - q)) return false;
    u.Uc = (int32_t)(csz / 8);
    u.ucnt_off = q + 8;
    q += 8 + (int64_t)csz;
    if (!need(8)) return false;
    const uint64_t psz = ld_u64(in + q);
    if ((psz & 7) || psz > (uint64_t)(end - q)) return false;
    u.P = (int32_t)(psz / 8);
    u.pair_off = q + 8;
    q += 8 + (int64_t)psz;
    if (q > end) return false;
    // Every per-unit scratch row holds M + 1 words: the sections that are expanded into one
    // (with_previous, unmatched ids, pairs) must fit it, and the sections indexed by matched
    // row or run (matched_index, unmatched counts) must cover what the later kernels read.
    if (u.M < 0 || u.P > u.M || u.W > u.M || (int64_t)u.U > (int64_t)u.M + 1 || (u.Uc > 0 && u.Uc != u.U) ||
        (u.Mi > 0 && u.Mi != u.M))
      return false;
    if (k >= max_units) return false;
    if (units) units[first_unit + k] = u;
    k++;
  }
  *count = k;
  return q == end;
}

__global__ void __launch_bounds__(64) k_dec_units(const uint8_t* __restrict__ in, const DChunk* __restrict__ chunks,
                                                  int32_t n_chunks, const int32_t* __restrict__ first_unit,
                                                  int32_t* __restrict__ nunits, DUnit* __restrict__ units, uint32_t* err) {
  latency_kernel();
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= n_chunks) return;
  int32_t k = 0;
  if (!walk_units(in, chunks[c], units ? first_unit[c] : 0, units, &k)) raise_error(err, kErrCorrupt);
  if (nunits) nunits[c] = k;
}

// One chunk payload at `in` (len bytes), everything on the device: the unit table (at most
// max_units entries, the rest zeroed so that fixed-size launches over max_units units find
// empty units), the scratch offsets of each unit, an identity launch order and the header
// words {error bits, units, window-tier failures, list-tier failures, matched events (2
// words)}.  A payload whose units need more than max_rows scratch rows (sum of M + 1) or more
// than perm_capacity permutation entries is refused with the limit bit and an empty table.
__global__ void __launch_bounds__(64) k_dec_chunk_units(const uint8_t* __restrict__ in, int64_t len, int32_t max_units,
                                                        int64_t max_rows, int64_t perm_capacity,
                                                        int32_t* __restrict__ hdr, int32_t* __restrict__ order,
                                                        DUnit* __restrict__ units) {
  latency_kernel();
  __shared__ int32_t nu_s;
  if (threadIdx.x == 0) {
    int32_t k = 0;
    uint32_t e = 0;
    const DChunk c{0, len, 0, 0};
    if ((len & 7) || len <= 0 || !walk_units(in, c, 0, units, &k, max_units)) {
      e |= 1u << kErrCorrupt;
      k = 0;
    }
    int64_t wb = 0, ko = 0;
    for (int32_t q = 0; q < k; q++) {
      DUnit& u = units[q];
      u.wbase = wb;
      u.rec_off = ko + q;  // not used by the permutation kernels
      u.key_off = ko;
      u.fb = 1;  // whole-unit tiers only
      u.nseg = 1;
      u.seg0 = q;
      wb += (int64_t)u.M + 1;
      ko += u.M;
    }
    if (wb > max_rows || ko > perm_capacity) {
      e |= 1u << kErrLimit;
      k = 0;
      ko = 0;
    }
    hdr[0] = (int32_t)e;
    hdr[1] = k;
    hdr[2] = 0;
    hdr[3] = 0;
    hdr[4] = (int32_t)(ko & 0xffffffff);
    hdr[5] = (int32_t)(ko >> 32);
    nu_s = k;
  }
  __syncthreads();
  const int32_t nu = nu_s;
  for (int32_t q = threadIdx.x; q < max_units; q += 64) {
    order[q] = q;
    if (q >= nu) units[q] = DUnit{};
  }
}

// Inverse LP of one section: x = prefix(prefix(y)) mod 2^64.  Loads either 8-byte words
// or sign-extended int32 (the pair sections, rempi_copy_vec_int :1004-1014).
template <bool I32>
__device__ void inverse_lp(const uint8_t* __restrict__ src, int32_t n, uint64_t* __restrict__ dst, uint64_t* lds) {
  uint64_t cz = 0, cx = 0;
  for (int32_t b = 0; b < n; b += 256) {
    const int32_t i = b + threadIdx.x;
    uint64_t y = 0;
    if (i < n) y = I32 ? sext((int32_t)ld_u32(src + 4 * (int64_t)i)) : ld_u64(src + 8 * (int64_t)i);
    uint64_t tz, tx;
    const uint64_t zl = block_exclusive_scan<256>(y, (uint64_t)0, OpAdd(), lds, &tz) + y;
    const uint64_t z = (i < n) ? zl + cz : 0;
    const uint64_t xl = block_exclusive_scan<256>(z, (uint64_t)0, OpAdd(), lds, &tx) + z;
    if (i < n) dst[i] = xl + cx;
    cx += tx;
    cz += tz;
  }
}

// with_previous and unmatched-id sections (the pair sections are inverted by the
// permutation kernel as it consumes them).  Also: the with_next flag of every matched row
// (with_previous_bool_vec, :1104-1110; wnf must be zeroed) and the unmatched-id checks of
// the records stage (ids strictly increasing and <= count), so that later kernels can
// binary-search the id list.
__global__ void __launch_bounds__(256) k_dec_sections(const DUnit* __restrict__ units, const uint8_t* __restrict__ in,
                                                      uint64_t* __restrict__ wpd, uint64_t* __restrict__ uidd,
                                                      uint8_t* __restrict__ wnf, uint32_t* err) {
  __shared__ uint64_t lds[4];
  const DUnit u = units[blockIdx.x];
  inverse_lp<false>(in + u.wp_off, u.W, wpd + u.wbase, lds);
  inverse_lp<false>(in + u.uid_off, u.U, uidd + u.wbase, lds);
  __syncthreads();
  for (int32_t k = threadIdx.x; k < u.W; k += 256) {
    const uint64_t w = wpd[u.wbase + k];
    if (w >= (uint64_t)u.M) raise_error(err, kErrCorrupt);
    else wnf[u.wbase + w] = 1;
  }
  if (u.Uc > 0) {
    const uint64_t* ids = uidd + u.wbase;
    for (int32_t k = threadIdx.x; k < u.U; k += 256)
      if (ids[k] > (uint64_t)u.M || (k > 0 && ids[k] <= ids[k - 1])) raise_error(err, kErrCorrupt);
  }
}

// cdc_prepare_decode_indices, one lane per unit: the list 0..M-1 (+ sentinel M, circular
// as std::list), each pair moves `id` `delay` nodes past its old successor.
__global__ void __launch_bounds__(64) k_dec_perm_lane(const DUnit* __restrict__ units, int32_t n_units,
                                                      const uint64_t* __restrict__ idd, const uint64_t* __restrict__ dld,
                                                      int32_t* __restrict__ nx, int32_t* __restrict__ pv,
                                                      int32_t* __restrict__ perm, uint32_t* err) {
  const int ui = blockIdx.x * 64 + threadIdx.x;
  if (ui >= n_units) return;
  const DUnit u = units[ui];
  if (u.fb != 3) return;  // rebuilt by an earlier tier
  const int32_t M = u.M;
  int32_t* n = nx + u.wbase;
  int32_t* p = pv + u.wbase;
  for (int32_t i = 0; i <= M; i++) {
    n[i] = (i == M) ? 0 : i + 1;
    p[i] = (i == 0) ? M : i - 1;
  }
  for (int32_t k = 0; k < u.P; k++) {
    const int32_t id = (int32_t)idd[u.wbase + k];
    int32_t dl = (int32_t)dld[u.wbase + k];
    if (id < 0 || id >= M || dl > M || dl < -M) {
      raise_error(err, kErrCorrupt);
      return;
    }
    int32_t at = n[id];
    n[p[id]] = n[id];
    p[n[id]] = p[id];
    for (; dl > 0; dl--) at = n[at];
    for (; dl < 0; dl++) at = p[at];
    const int32_t before = p[at];
    n[before] = id;
    p[id] = before;
    n[id] = at;
    p[at] = id;
  }
  int32_t q = n[M];
  int32_t* pm = perm + u.key_off;
  for (int32_t i = 0; i < M; i++, q = n[q]) {
    if (q < 0 || q >= M) { raise_error(err, kErrCorrupt); return; }
    pm[q] = i;
  }
}

// ---------------------------------------------------------------------------------------
// Permutation rebuild, one wave per unit, exact.
//
// The list of cdc_prepare_decode_indices is kept as three parts: a settled prefix (already
// written to perm), a window of W = 64*K slots held across the wave's lanes (slot s in
// register s/64 of lane s%64), and the untouched suffix nu..M-1 (still the identity).
// Every pair is uniform across the wave: pull the suffix up to its id, find it (ballots),
// close the gap (lane shift), step `delay` slots, open a gap and insert (lane shift).  The
// window's head is settled only when the window is full.  A move that would reach into
// the settled prefix marks the unit for the next attempt (larger K, then the sequential
// k_dec_perm_lane); everything written so far is overwritten by that attempt.
namespace {

template <int K>
struct Window {
  int32_t v[K];  // v[j] = slot 64*j + lane

  // position of value x among the first n slots, or -1 (uniform)
  __device__ __forceinline__ int32_t find(int32_t x, int32_t n) const {
    const int l = lane_id();
#pragma unroll
    for (int j = 0; j < K; j++) {
      const uint64_t m = __builtin_amdgcn_ballot_w64(v[j] == x && 64 * j + l < n);
      if (m) return 64 * j + (int32_t)__ffsll((unsigned long long)m) - 1;
    }
    return -1;
  }
  // slots >= p take the value of slot +1 (p uniform)
  __device__ __forceinline__ void close_gap(int32_t p) {
    const int l = lane_id();
#pragma unroll
    for (int j = 0; j < K; j++) {
      // DPP wave_shl:1 -- lane l reads lane l+1 (no LDS round trip)
      int32_t nx = __builtin_amdgcn_update_dpp(0, v[j], 0x130, 0xf, 0xf, false);
      if (j + 1 < K) {
        const int32_t wrap = __builtin_amdgcn_readlane(v[j + 1], 0);
        if (l == 63) nx = wrap;
      }
      if (64 * j + l >= p) v[j] = nx;
    }
  }
  // slots > t take the value of slot -1, slot t = x
  __device__ __forceinline__ void open_gap(int32_t t, int32_t x) {
    const int l = lane_id();
    int32_t carry = 0;
#pragma unroll
    for (int j = 0; j < K; j++) {
      // DPP wave_shr:1 -- lane l reads lane l-1
      int32_t pv = __builtin_amdgcn_update_dpp(0, v[j], 0x138, 0xf, 0xf, false);
      const int32_t last = __builtin_amdgcn_readlane(v[j], 63);
      if (l == 0) pv = carry;
      carry = last;
      const int32_t s = 64 * j + l;
      if (s > t) v[j] = pv;
      else if (s == t) v[j] = x;
    }
  }
  // drop the first e slots (e uniform, 0 < e < 64*K)
  __device__ __forceinline__ void shift_out(int32_t e) {
    const int l = lane_id();
    int32_t nv[K];
#pragma unroll
    for (int j = 0; j < K; j++) {
      const int32_t src = 64 * j + l + e;  // source slot
      int32_t r = 0;
#pragma unroll
      for (int q = 0; q < K; q++) {
        const int32_t got = __shfl(v[q], src & 63, 64);
        if ((src >> 6) == q) r = got;
      }
      nv[j] = r;
    }
#pragma unroll
    for (int j = 0; j < K; j++) v[j] = nv[j];
  }
};

}  // namespace

template <int K>
__global__ void __launch_bounds__(64) k_dec_perm_window(DUnit* __restrict__ units, int32_t n_units, int32_t want_fb,
                                                        const uint64_t* __restrict__ idd, const uint64_t* __restrict__ dld,
                                                        int32_t* __restrict__ perm, int32_t* __restrict__ nfail) {
  constexpr int32_t W = 64 * K;
  DUnit& u = units[blockIdx.x];
  if (u.fb != want_fb) return;
  const int l = lane_id();
  const int32_t M = u.M, P = u.P;
  int32_t* pm = perm + u.key_off;
  Window<K> win;
#pragma unroll
  for (int j = 0; j < K; j++) win.v[j] = -1;
  int32_t wl = 0, nu = 0, settled = 0;
  bool fail = false;
  auto evict = [&](int32_t e) {  // settle the first e slots
#pragma unroll
    for (int j = 0; j < K; j++)
      if (64 * j + l < e) pm[win.v[j]] = settled + 64 * j + l;
    win.shift_out(e);
    settled += e;
    wl -= e;
  };
  auto pull = [&](int32_t upto) {  // append suffix elements nu..upto-1 (evicting as needed)
    while (nu < upto) {
      int32_t cnt = min(upto - nu, W - wl);
      if (cnt == 0) {
        evict(min(wl, W / 2));
        continue;
      }
#pragma unroll
      for (int j = 0; j < K; j++) {
        const int32_t s = 64 * j + l;
        if (s >= wl && s < wl + cnt) win.v[j] = nu + (s - wl);
      }
      wl += cnt;
      nu += cnt;
    }
  };
  for (int32_t k0 = 0; k0 < P && !fail; k0 += 64) {
    const int32_t idv = (k0 + l < P) ? (int32_t)idd[u.wbase + k0 + l] : 0;
    const int32_t dlv = (k0 + l < P) ? (int32_t)dld[u.wbase + k0 + l] : 0;
    const int32_t nk = min(64, P - k0);
    for (int32_t q = 0; q < nk; q++) {
      const int32_t x = __builtin_amdgcn_readlane(idv, q);
      const int32_t d = __builtin_amdgcn_readlane(dlv, q);
      if (x < 0 || x >= M) { fail = true; break; }
      if (x >= nu) pull(x + 1);
      const int32_t px = win.find(x, wl);
      if (px < 0) { fail = true; break; }  // already settled
      win.close_gap(px);
      wl--;
      int32_t t = px + d;
      if (t < 0) { fail = true; break; }
      while (wl < t) {  // bring the suffix in up to the target slot
        if (wl == W) {
          const int32_t e = min(W / 2, t);
          evict(e);
          t -= e;
          continue;
        }
        const int32_t cnt = min(t - wl, W - wl);
        if (nu + cnt > M) { fail = true; break; }
#pragma unroll
        for (int j = 0; j < K; j++) {
          const int32_t s = 64 * j + l;
          if (s >= wl && s < wl + cnt) win.v[j] = nu + (s - wl);
        }
        wl += cnt;
        nu += cnt;
      }
      if (fail) break;
      if (wl == W) {
        if (t == 0) {  // x goes right after the settled prefix: settle it directly
          if (l == 0) pm[x] = settled;
          settled++;
          continue;
        }
        evict(1);
        t -= 1;
      }
      win.open_gap(t, x);
      wl++;
    }
  }
  if (fail) {
    if (l == 0) {
      u.fb = want_fb + 1;
      atomicAdd(nfail, 1);
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < K; j++)
    if (64 * j + l < wl) pm[win.v[j]] = settled + 64 * j + l;
  settled += wl;
  for (int32_t v = nu + l; v < M; v += 64) pm[v] = settled + (v - nu);
}

template __global__ void k_dec_perm_window<2>(DUnit*, int32_t, int32_t, const uint64_t*, const uint64_t*, int32_t*, int32_t*);
template __global__ void k_dec_perm_window<4>(DUnit*, int32_t, int32_t, const uint64_t*, const uint64_t*, int32_t*, int32_t*);

// ---------------------------------------------------------------------------------------
// Pair sections of every unit in one pass, one workgroup per unit: the inverse linear
// prediction of ids and delays (x = prefix(prefix(y)) of the sign-extended int32 words, mod
// 2^64, decode :1004-1014 + rempi_compression_util.cpp:157-168), and from it
//   mode & 1: the unit's pair segments (DSeg) -- the prediction state at the first replayed pair
//             of every segment (pcar: z, x of ids, z, x of delays before that pair) and the list
//             positions each segment owns, from the suffix minima of the ids;
//   mode & 2: the decoded pair arrays of the units that left the first tier (fb != 0);
//   mode & 4: the decoded pair arrays of every unit (table dumps).
namespace {
__device__ __forceinline__ int32_t seg_floor(int32_t min_id) { return max(0, min_id - kSegDelta) & ~15; }
}  // namespace

// One wave per unit and no workgroup barrier: a unit's pairs are one chain of prefix sums, 256
// pairs per round (four per lane, the next round's words already in flight), and a wave on its
// own is not held up by the other waves of a workgroup when the GPU is busy with other streams.
__global__ void __launch_bounds__(64) k_dec_pair_scan(const DUnit* __restrict__ units, const uint8_t* __restrict__ in,
                                                      int32_t mode, DSeg* __restrict__ segs, int64_t* __restrict__ pcar,
                                                      uint64_t* __restrict__ idd, uint64_t* __restrict__ dld) {
  __shared__ int32_t bmin[kSegMaxP / kSegWarm + 1];  // smallest id of every kSegWarm pairs, then suffix minima
  const int32_t ui = blockIdx.x;
  const DUnit u = units[ui];
  const int32_t P = u.P, l = threadIdx.x;
  const bool lists = (mode & 1) && u.nseg > 1;  // (more than one segment: P <= kSegMaxP)
  const bool store = (mode & 4) || ((mode & 2) && u.fb != 0);
  if ((mode & 1) && u.nseg <= 1 && l == 0) segs[u.seg0] = DSeg{ui, 0, 0, P, 0, kSegNoCap, 0, 0};
  if (!lists && !store) return;
  const int32_t* yid = reinterpret_cast<const int32_t*>(in + u.pair_off);
  const int32_t* ydl = yid + P;
  uint64_t czi = 0, cxi = 0, czd = 0, cxd = 0;  // z, x before the round's first pair
  int32_t wi[4], wd[4];
  auto load = [&](int32_t k) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      wi[q] = (k + q < P) ? yid[k + q] : 0;
      wd[q] = (k + q < P) ? ydl[k + q] : 0;
    }
  };
  load(4 * l);
  for (int32_t t0 = 0; t0 < P; t0 += 256) {
    const int32_t k = t0 + 4 * l;
    uint64_t zi[4], zd[4], s2i = 0, s2d = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      zi[q] = (q ? zi[q - 1] : 0) + sext(wi[q]);
      zd[q] = (q ? zd[q - 1] : 0) + sext(wd[q]);
      s2i += zi[q];
      s2d += zd[q];
    }
    load(k + 256);  // (in flight during the scans)
    const uint64_t zni = wave_inclusive_scan(zi[3], OpAdd()), znd = wave_inclusive_scan(zd[3], OpAdd());
    const uint64_t zoi = zni - zi[3], zod = znd - zd[3];
    const uint64_t ai = 4 * zoi + s2i, ad = 4 * zod + s2d;
    const uint64_t xni = wave_inclusive_scan(ai, OpAdd()), xnd = wave_inclusive_scan(ad, OpAdd());
    const uint64_t z0i = czi + zoi, z0d = czd + zod;
    uint64_t xi = cxi + 4 * czi * (uint64_t)l + (xni - ai), xd = cxd + 4 * czd * (uint64_t)l + (xnd - ad);
    constexpr int32_t kPer = kSegPairs / kSegWarm;
    if (lists && (k & (kSegWarm - 1)) == 0 && (k / kSegWarm) % kPer == kPer - 1) {  // k = s * kSegPairs - kSegWarm
      const int32_t sg = (k / kSegWarm + 1) / kPer;
      if (sg < u.nseg) {
        int64_t* o = pcar + 4 * (u.seg0 + sg);
        o[0] = (int64_t)z0i;
        o[1] = (int64_t)xi;
        o[2] = (int64_t)z0d;
        o[3] = (int64_t)xd;
      }
    }
    int32_t mn = INT32_MAX;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      xi += z0i + zi[q];
      xd += z0d + zd[q];
      if (k + q < P) {
        if (store) {
          idd[u.wbase + k + q] = xi;
          dld[u.wbase + k + q] = xd;
        }
        mn = min(mn, (int32_t)xi);
      }
    }
    if (lists) {
#pragma unroll
      for (int dlt = 16; dlt >= 1; dlt >>= 1) mn = min(mn, __shfl_xor(mn, dlt, 64));
      if ((l & 31) == 0) bmin[(t0 >> 7) + (l >> 5)] = mn;
    }
    cxi += 256 * czi + __shfl(xni, kWave - 1, kWave);
    cxd += 256 * czd + __shfl(xnd, kWave - 1, kWave);
    czi += __shfl(zni, kWave - 1, kWave);
    czd += __shfl(znd, kWave - 1, kWave);
  }
  if (!lists) return;
  const int32_t nb = (P + kSegWarm - 1) / kSegWarm;
  int32_t carry = INT32_MAX;  // suffix minima, 64 entries at a time from the top
  for (int32_t hi = nb; hi > 0; hi -= kWave) {
    const int32_t idx = hi - 1 - l;
    int32_t v = idx >= 0 ? bmin[idx] : INT32_MAX;
    v = min(wave_inclusive_scan(v, OpMin()), carry);
    if (idx >= 0) bmin[idx] = v;
    carry = __shfl(v, kWave - 1, kWave);
  }
  for (int32_t sg = l; sg < u.nseg; sg += kWave) {
    const int32_t ka = sg * kSegPairs;
    DSeg d;
    d.unit = ui;
    d.s = sg;
    d.ka = ka;
    d.ke = min(P, ka + kSegPairs);
    d.own = sg ? seg_floor(bmin[ka / kSegWarm]) : 0;
    d.cap = sg + 1 < u.nseg ? min(kSegNoCap, seg_floor(bmin[(ka + kSegPairs) / kSegWarm])) : kSegNoCap;
    d.base0 = sg ? seg_floor(bmin[(ka - kSegWarm) / kSegWarm]) : 0;
    d.pad = 0;
    segs[u.seg0 + sg] = d;
  }
}

// ---------------------------------------------------------------------------------------
// Permutation rebuild in 16-lane groups (four per wave): one pair segment per group (SEG, the
// first tier) or one whole unit per group (the second tier, for units whose segments did not
// check out).
//
// The list is held as a window of list positions [base, base + W) in a per-group LDS ring,
// plus an LDS map from an element's low bits to the ring slot it was last put in (one byte
// per entry: the LDS a group needs decides how many groups a CU holds, and the rebuild is
// bound by the latency of its dependent steps, not by issue).  An entry is a hint: the slot's
// content says whether the element is there, so stale and colliding entries cost a failed
// look-up (the unit goes to the next tier), never a wrong move.  Every position at
// or past the window still holds its initial element (position q holds q): nothing has
// been moved there.  A pair moves x from its position p to t = p + delay of the list
// without x, i.e. rotates the window slots between p and t by one: one LDS read + write
// per 16 slots across the group's lanes, and the moved elements are re-pointed in the map.
// The window slides forward 16 positions at a time (the front 16 are settled into perm and
// its inverse cinv); sliding is a base increment, nothing moves.
//
// Why groups: with one unit per wave the per-pair control is scalar code (~40 SALU per
// pair) and the scalar unit is shared by the CU's four SIMDs, so that version is bound by
// scalar issue; here the per-pair control is group-uniform vector code shared by four
// groups.  All groups consume one pair per step (the pair index is the step count), so the
// q-th pair of a 16-pair batch is broadcast from group lane q with DPP row_newbcast.
//
// Segments.  One unit's pair list is one dependency chain (17 K pairs in the bench traces),
// and a batch has too few units to fill the GPU with such chains.  But a move only touches
// the list near its id, and ids rise along the pair list, so the state a stretch of pairs
// meets depends on the pairs shortly before it only.  A segment therefore starts from the
// untouched list, replays the kSegWarm pairs before its own without writing anything (a pair
// that does not fit the window is skipped there), moves its window to the first position it
// owns (`own`) and writes the kSegWin positions from there to dumpW.  Its predecessor never
// slides past that position (`cap`) and writes the same positions of its final state to
// dumpT; behind them both lists are untouched.  k_dec_perm_check compares the two: where they
// agree the segment started from the list the sequential replay has at that pair, and since it
// fails (like the whole-unit tier) on any move that reaches below its window, everything it
// wrote is what the sequential replay writes.  A unit with a failed or disagreeing segment
// goes to the next tier whole; every tier rewrites all outputs of the units it takes.
//
// A pair that reaches behind the window, an element no longer in it, or a step past the
// list end (the std::list wrap through its sentinel) fails the group's unit for this tier.
namespace {
constexpr int32_t kGW = kSegWin;  // window slots per group (power of two)
constexpr int32_t kGMap = 256;    // element map entries per group (power of two)
constexpr int32_t kGAhead = 56;   // an untouched x is brought to >= kGAhead slots before the end

template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

__device__ __forceinline__ int64_t row_incl_scan64(int64_t v) {  // inclusive scan over a 16-lane row
  const int j = threadIdx.x & 15;
#pragma unroll
  for (int d = 1; d < 16; d <<= 1) {
    const int64_t o = __shfl_up(v, d, 16);
    if (j >= d) v += o;
  }
  return v;
}

template <int Q>
__device__ __forceinline__ int32_t row_bcast(int32_t v) {
  // row_newbcast:Q (every lane has a source: bound_ctrl only spares the copy of an old value)
  return __builtin_amdgcn_update_dpp(0, v, 0x150 + Q, 0xf, 0xf, true);
}

// Lane masks of a compare, straight from v_cmp into a scalar register pair (LLVM integer
// predicates), and a lane's own bit of such a mask as a select condition.
using mask64 = unsigned long long;
__device__ __forceinline__ mask64 m_lt(int32_t x, int32_t y) { return __builtin_amdgcn_sicmp(x, y, 40); }
__device__ __forceinline__ mask64 m_le(int32_t x, int32_t y) { return __builtin_amdgcn_sicmp(x, y, 41); }
__device__ __forceinline__ mask64 m_gt(int32_t x, int32_t y) { return __builtin_amdgcn_sicmp(x, y, 38); }
__device__ __forceinline__ mask64 m_ge(int32_t x, int32_t y) { return __builtin_amdgcn_sicmp(x, y, 39); }
__device__ __forceinline__ mask64 m_ne(int32_t x, int32_t y) { return __builtin_amdgcn_sicmp(x, y, 33); }
__device__ __forceinline__ mask64 mu_ge(uint32_t x, uint32_t y) { return __builtin_amdgcn_uicmp(x, y, 35); }
__device__ __forceinline__ bool lane_of(mask64 m) { return __builtin_amdgcn_inverse_ballot_w64(m); }
}  // namespace

template <int MODE>  // 0: whole units (`order`), 1: all segments, 2: the segments listed in `order` again, from dumpT
__global__ void __launch_bounds__(64) k_dec_perm_seg(DUnit* __restrict__ units, const int32_t* __restrict__ order,
                                                     const DSeg* __restrict__ segs, int64_t n_items, int32_t want_fb,
                                                     const uint8_t* __restrict__ in, const int64_t* __restrict__ pcar,
                                                     int32_t* __restrict__ perm, int32_t* __restrict__ cinv,
                                                     int32_t* __restrict__ dumpT, int32_t* __restrict__ dumpW,
                                                     int32_t* __restrict__ nfail) {
  constexpr int32_t W = kGW, WM = kGW - 1, MM = kGMap - 1;
  __shared__ int32_t win_all[4][W + 16];      // + one dummy slot per lane
  __shared__ uint8_t emap_all[4][kGMap + 16];  // ring slot of the element with these low bits; + dummies
  const int g = threadIdx.x >> 4, j = threadIdx.x & 15;
  int32_t* win = win_all[g];
  uint8_t* emap = emap_all[g];
  constexpr bool SEG = MODE != 0, REDO = MODE == 2;
  int64_t gi = (int64_t)blockIdx.x * 4 + g;
  int32_t ui = -1;
  DSeg sd{-1, 0, 0, 0, 0, kSegNoCap, 0, 0};
  if (REDO) {  // order[0]: entries listed (may exceed the list's n_items slots), order[1 + k]: segment
    const int64_t k = gi;
    gi = -1;
    if (k < min((int64_t)order[0], n_items)) {
      gi = order[1 + k];
      sd = segs[gi];
      ui = sd.unit;
    }
  } else if (gi < n_items) {
    if (SEG) {
      sd = segs[gi];
      ui = sd.unit;
    } else {
      ui = order[gi];
    }
  }
  int32_t M = 0, Pu = 0;
  int64_t key_off = 0, pair_off = 0;
  bool sim = false;  // the group's unit is at this tier
  if (ui >= 0) {
    const DUnit& u = units[ui];
    sim = (u.fb == want_fb);
    M = u.M;
    Pu = u.P;
    key_off = u.key_off;
    pair_off = u.pair_off;
    if (!SEG) sd.ke = Pu;
  }
  const bool wact = SEG && sim && sd.s > 0;            // replays kSegWarm pairs first
  const mask64 wactm = __builtin_amdgcn_ballot_w64(wact);
  const bool hasn = SEG && sd.cap != kSegNoCap;        // a segment follows: leave it the final state
  const int32_t ka = sd.ka, ke = sim ? sd.ke : sd.ka;  // the group's own pairs
  const int32_t klo = wact ? ka - kSegWarm : ka;       // first pair it reads
  const int32_t own = sd.own, cap = sd.cap;
  int32_t* pm = perm + key_off;
  int32_t* ci = cinv + key_off;
  const int32_t* yid = reinterpret_cast<const int32_t*>(in + pair_off);
  const int32_t* ydl = yid + Pu;
  int64_t czi = 0, cxi = 0, czd = 0, cxd = 0;  // inverse-LP carries (rempi_compression_util.cpp:157-168)
  if (wact) {
    const int64_t* o = pcar + 4 * gi;
    czi = o[0];
    cxi = o[1];
    czd = o[2];
    cxd = o[3];
  }
  int32_t base = sd.base0;  // (a multiple of 16)
  for (int32_t q = j; q < W; q += 16) {  // (map entries of elements outside the window: never trusted, see step)
    const int32_t e = base + q;
    win[e & WM] = e;
    emap[e & MM] = (uint8_t)(e & WM);
  }
  // Flags of a step are wave-uniform lane masks in scalar registers (group-uniform conditions
  // set all 16 bits of a group): combining and testing them is scalar work, and a lane reads
  // its bit straight from the mask as a select operand.
  mask64 failm = ~__builtin_amdgcn_ballot_w64(sim);  // groups that take no (more) pairs at this tier
  auto slide = [&](auto warm_c, mask64 gom) {  // settle [base, base+16), open [base+W, base+W+16) as identity
    constexpr bool WARM = decltype(warm_c)::value;
    const bool go = lane_of(gom);
    const int32_t ph = go ? ((base + j) & WM) : W + j;
    const int32_t v = win[ph];  // (dummy slot when not sliding)
    if (!WARM) {
      if (go && v < M) {
        pm[v] = base + j;
        ci[base + j] = v;
      }
    }
    const int32_t e = base + W + j;
    __builtin_amdgcn_wave_barrier();
    win[ph] = e;
    emap[go ? (e & MM) : kGMap + j] = (uint8_t)ph;  // (e's ring slot is the one just settled)
    base += go ? 16 : 0;
  };
  // one pair of all four groups: x, d group-uniform.  WARM: the replay before a segment's own
  // pairs -- the window stays at or below `own`, nothing is written, and a pair that does not
  // fit is skipped (the state is checked afterwards).  Otherwise the window stays at or below
  // `cap` and a pair that does not fit fails the unit.
  auto step = [&](auto warm_c, mask64 in_m, int32_t x, int32_t d) {
      constexpr bool WARM = decltype(warm_c)::value;
      const int32_t lim = WARM ? own : cap;
      // Common path without divergent branches: predicated selects, LDS accesses of
      // inactive lanes go to per-lane dummy slots; rare cases (slides, targets past the
      // window, rotations longer than 16 slots) take wave-uniform detours.
      // (an id outside [0, M) has failed the unit when its batch was formed, in lp())
      mask64 actm = in_m & ~failm;
      // an untouched x (at position x) is brought kGAhead slots before the window end
      const mask64 farm = actm & m_ge(x, base + W);
      if (farm)
        while (true) {
          const mask64 gom = farm & m_ge(x, base + W - kGAhead) & m_le(base + 16, lim);
          if (!gom) break;
          slide(warm_c, gom);
        }
      // the map gives a ring slot; x is there or the entry is stale (another element with the
      // same low bits, or none): the slot's content decides, read beside the rotation's first
      // read below, so that the check costs no LDS round trip of its own
      const int32_t slot = emap[lane_of(actm) ? (x & MM) : kGMap + j] & WM;
      int32_t p = (slot - base) & WM;
      int32_t t = p + d;
      const mask64 badm = actm & (m_lt(t, 0) | m_gt(base + t, M - 1));
      if (!WARM) failm |= badm;
      actm &= ~badm;
      auto in_slot = [&]() {  // drops the groups whose x is not in `slot`
        int32_t chk = win[lane_of(actm) ? slot : W + j];
        asm volatile("" : "+v"(chk));
        const mask64 missm = actm & m_ne(chk, x);
        if (!WARM) failm |= missm;
        actm &= ~missm;
      };
      mask64 overm = actm & m_gt(t, W - 1);
      if (overm) {
        in_slot();  // (before the window moves on account of x)
        overm &= actm;
        while (overm) {
          const mask64 stuckm = overm & (m_lt(p, 16) | m_gt(base + 16, lim));
          if (!WARM) failm |= stuckm;
          actm &= ~stuckm;
          const mask64 slm = overm & ~stuckm;
          slide(warm_c, slm);
          const int32_t back = lane_of(slm) ? 16 : 0;
          p -= back;
          t -= back;
          overm = actm & m_gt(t, W - 1);
        }
      }
      // rotation of the slots between p and t, 16 at a time
      const bool fwd = t >= p;
      const int32_t len = fwd ? t - p : p - t;
      const int32_t dir = fwd ? 1 : -1;
      auto chunk = [&](int32_t c) {
        const int32_t o = c + j;
        const mask64 ltm = m_lt(o, len);
        const int32_t s = p + dir * o;
        const int32_t rd = lane_of(actm & ltm) ? ((base + s + dir) & WM) : W + j;
        int32_t w = win[rd];
        asm volatile("" : "+v"(w));  // keep the read unconditional (no exec-mask branch around it)
        if (c == 0) in_slot();
        const bool sel = lane_of(actm & m_le(o, len));
        const int32_t v = lane_of(ltm) ? w : x;
        const int32_t ws = (base + s) & WM;
        __builtin_amdgcn_wave_barrier();
        win[sel ? ws : W + j] = v;
        emap[sel ? (v & MM) : kGMap + j] = (uint8_t)ws;
        __builtin_amdgcn_wave_barrier();
      };
      chunk(0);
      if (actm & m_ge(len, 16))
        for (int32_t c = 16; actm & m_le(c, len); c += 16) chunk(c);
  };
  // 16 pairs at a time: inverse LP of the raw words (x = prefix(prefix(y)) of the
  // sign-extended int32 sections, mod 2^64, decode :1004-1014 + :157-168; the sim uses the
  // low 32 bits), then the steps, each taking group lane 0 (row_newbcast:0) and shifting
  // the batch down a lane
  int32_t xs = 0, ds = 0;
  auto lp = [&](auto warm_c, int32_t k0, int32_t yw_i, int32_t yw_d) {
    constexpr bool WARM = decltype(warm_c)::value;
    const int64_t yi = (int64_t)yw_i, yd = (int64_t)yw_d;
    const int64_t zi = row_incl_scan64(yi), zd = row_incl_scan64(yd);
    const int64_t xi = cxi + (int64_t)(j + 1) * czi + row_incl_scan64(zi);
    const int64_t xd = cxd + (int64_t)(j + 1) * czd + row_incl_scan64(zd);
    czi += __shfl(zi, 15, 16);
    czd += __shfl(zd, 15, 16);
    cxi = __shfl(xi, 15, 16);
    cxd = __shfl(xd, 15, 16);
    xs = (int32_t)xi;
    ds = (int32_t)xd;
    if (!WARM) {
      // an id outside [0, M) among the batch's pairs fails the unit (for this tier) at once
      const bool inb = k0 + j >= ka && k0 + j < ke;
      const uint64_t badm = __builtin_amdgcn_ballot_w64(inb && (uint32_t)xs >= (uint32_t)M);
      failm |= m_ne((int32_t)((badm >> (threadIdx.x & 48)) & 0xffffu), 0);
    }
  };
  auto steps = [&](auto warm_c, int32_t k0, int32_t nq) {
    constexpr bool WARM = decltype(warm_c)::value;
    for (int32_t q = 0; q < nq; q++) {
      const int32_t x = row_bcast<0>(xs), d = row_bcast<0>(ds);
      xs = __builtin_amdgcn_update_dpp(xs, xs, 0x101, 0xf, 0xf, false);  // row_shl:1
      ds = __builtin_amdgcn_update_dpp(ds, ds, 0x101, 0xf, 0xf, false);
      step(warm_c, WARM ? wactm : m_lt(k0 + q, ke), x, d);
    }
  };
  // Two batches per round.  The raw words of a batch are loaded one batch ahead, and each
  // load is issued only after the previous wait (the compiler waits for all outstanding
  // memory operations at every use), so a wait never covers a load issued just before it.
  auto ld = [&](const int32_t* y, int32_t k) { return (k + j >= klo && k + j < ke) ? y[k + j] : 0; };
  const std::integral_constant<bool, true> warm_t{};
  const std::integral_constant<bool, false> main_t{};
  int32_t ai, ad, bi, bd;
  if (SEG && wactm) {
    const int32_t kb = ka - kSegWarm;  // (groups without a replay read nothing below ka: klo)
    ai = ld(yid, kb), ad = ld(ydl, kb), bi = ld(yid, kb + 16), bd = ld(ydl, kb + 16);
    for (int32_t i0 = 0; i0 < kSegWarm; i0 += 32) {
      lp(warm_t, kb + i0, ai, ad);
      ai = ld(yid, kb + i0 + 32);
      ad = ld(ydl, kb + i0 + 32);
      if (!REDO) steps(warm_t, kb + i0, 16);
      lp(warm_t, kb + i0 + 16, bi, bd);
      bi = ld(yid, kb + i0 + 48);
      bd = ld(ydl, kb + i0 + 48);
      if (!REDO) steps(warm_t, kb + i0 + 16, 16);
    }
    if (REDO) {
      // again, from the state the predecessor ended in (only the LP state came from the pairs
      // before): that state is now also the one this segment is on record as having started from
      if (wact) {
        base = own;
        for (int32_t q = j; q < W; q += 16) {
          const int32_t v = dumpT[gi * W + q];
          dumpW[gi * W + q] = v;
          win[(own + q) & WM] = v;
        }
        __builtin_amdgcn_wave_barrier();
        for (int32_t q = j; q < W; q += 16) {
          const int32_t v = win[(own + q) & WM];
          emap[v & MM] = (uint8_t)((own + q) & WM);
        }
      }
    } else {
      // the window moves up to the first owned position; the state there goes to the check
      for (mask64 gom; (gom = wactm & m_lt(base, own)) != 0;) slide(warm_t, gom);
      if (wact)
        for (int32_t q = j; q < W; q += 16) dumpW[gi * W + q] = win[(base + q) & WM];
    }
    if (!wact) {  // (a group without a replay went through it with zero words: nothing to carry over)
      czi = cxi = czd = cxd = 0;
    }
  } else {
    ai = ld(yid, ka), ad = ld(ydl, ka), bi = ld(yid, ka + 16), bd = ld(ydl, ka + 16);
  }
  const int32_t imax = __builtin_amdgcn_readfirstlane(wave_reduce(ke - ka, OpMax()));
  for (int32_t i0 = 0; i0 < imax; i0 += 32) {
    lp(main_t, ka + i0, ai, ad);
    ai = ld(yid, ka + i0 + 32);
    ad = ld(ydl, ka + i0 + 32);
    steps(main_t, ka + i0, min(16, imax - i0));
    if (i0 + 16 < imax) {
      lp(main_t, ka + i0 + 16, bi, bd);
      bi = ld(yid, ka + i0 + 48);
      bd = ld(ydl, ka + i0 + 48);
      steps(main_t, ka + i0 + 16, min(16, imax - i0 - 16));
    }
  }
  const bool fail = lane_of(failm);
  if (sim && fail && j == 0) {
    if (atomicCAS(&units[ui].fb, want_fb, want_fb + 1) == want_fb) atomicAdd(nfail, 1);
    if (SEG) atomicAdd(nfail + 4, 1);  // (diagnostics: segment runs that did not finish)
  }
  if (!fail) {
    const int32_t lim = min(M, cap);  // the positions below are this group's to write
    for (int32_t s = j; s < W; s += 16) {
      const int32_t v = win[(base + s) & WM];
      if (v < M && base + s < lim) {
        pm[v] = base + s;
        ci[base + s] = v;
      }
    }
    for (int32_t q = base + W + j; q < lim; q += 16) {
      pm[q] = q;
      ci[q] = q;
    }
    if (hasn)  // the state from `cap` on, for the next segment's check (base <= cap: the window never slid past it)
      for (int32_t q = j; q < W; q += 16) dumpT[(gi + 1) * W + q] = (cap + q < base + W) ? win[(cap + q) & WM] : cap + q;
  }
}

template __global__ void k_dec_perm_seg<0>(DUnit*, const int32_t*, const DSeg*, int64_t, int32_t, const uint8_t*,
                                           const int64_t*, int32_t*, int32_t*, int32_t*, int32_t*, int32_t*);
template __global__ void k_dec_perm_seg<1>(DUnit*, const int32_t*, const DSeg*, int64_t, int32_t, const uint8_t*,
                                           const int64_t*, int32_t*, int32_t*, int32_t*, int32_t*, int32_t*);
template __global__ void k_dec_perm_seg<2>(DUnit*, const int32_t*, const DSeg*, int64_t, int32_t, const uint8_t*,
                                           const int64_t*, int32_t*, int32_t*, int32_t*, int32_t*, int32_t*);

// The state a segment starts its own pairs from (dumpW) against the state its predecessor
// ends in (dumpT), kSegWin list positions from the segment's first owned one; 32 lanes per
// segment.  A segment that differs is listed in `redo` (redo[0] counts, redo[1..cap] hold the
// segments) and its unit marked in `redone`: k_dec_perm_seg<2> runs it again from dumpT, which
// is the sequential replay's state if the segments before it check out -- and the next check
// looks at all of them again.  The last check (`redo` null), or a full list, sends the unit to
// the next tier instead.  (A redone segment's earlier run may have written perm entries of
// elements that are not in its positions after all: k_dec_perm_inv rewrites perm of the marked
// units from cinv, which is indexed by position and so holds each segment's last run only.)
__global__ void __launch_bounds__(256) k_dec_perm_check(DUnit* __restrict__ units, const DSeg* __restrict__ segs,
                                                        int64_t nsegs, const int32_t* __restrict__ dumpT,
                                                        const int32_t* __restrict__ dumpW, int32_t* __restrict__ redo,
                                                        int32_t redo_cap, int32_t* __restrict__ redone,
                                                        int32_t* __restrict__ nfail) {
  static_assert(kSegWin == 128, "32 lanes x int4");
  const int64_t gi = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
  const int l = threadIdx.x & 31;
  bool diff = false;
  int32_t ui = -1;
  if (gi < nsegs) {
    const DSeg d = segs[gi];
    if (d.s > 0 && units[d.unit].fb == 0) {
      ui = d.unit;
      const int4 a = reinterpret_cast<const int4*>(dumpT)[gi * 32 + l], b = reinterpret_cast<const int4*>(dumpW)[gi * 32 + l];
      diff = a.x != b.x || a.y != b.y || a.z != b.z || a.w != b.w;
    }
  }
  const uint64_t m = __builtin_amdgcn_ballot_w64(diff);
  if (l == 0 && ui >= 0 && ((m >> (threadIdx.x & 32)) & 0xffffffffull)) {
    int32_t slot = redo_cap;
    if (redo) slot = atomicAdd(redo, 1);
    if (slot < redo_cap) {
      redo[1 + slot] = (int32_t)gi;
      redone[ui] = 1;
      atomicAdd(nfail + 5, 1);  // (diagnostics: segments run again)
    } else {
      if (atomicCAS(&units[ui].fb, 0, 1) == 0) atomicAdd(nfail, 1);
      atomicAdd(nfail + 6, 1);  // (diagnostics: segments that sent their unit on)
    }
  }
}

__global__ void __launch_bounds__(256) k_dec_perm_inv(const DUnit* __restrict__ units, const int32_t* __restrict__ redone,
                                                      const int32_t* __restrict__ cinv, int32_t* __restrict__ perm) {
  if (!redone[blockIdx.x]) return;
  const DUnit u = units[blockIdx.x];
  if (u.fb != 0) return;  // (a later tier rewrites both arrays)
  for (int32_t i = threadIdx.x; i < u.M; i += 256) perm[u.key_off + cinv[u.key_off + i]] = i;
}

// Rows whose permutation came from the fallback kernels: c = perm^-1.
__global__ void __launch_bounds__(256) k_dec_cinv(const DUnit* __restrict__ units, const int32_t* __restrict__ perm,
                                                  int32_t* __restrict__ cinv) {
  const DUnit u = units[blockIdx.x];
  if (u.fb == 0) return;
  for (int32_t v = threadIdx.x; v < u.M; v += 256) cinv[u.key_off + perm[u.key_off + v]] = v;
}

// Records reconstruction (decoded records as include/cdcx.h defines them), one block per 1024-row tile of a
// unit: matched row i is the event of clock order c_i (cinv, written by the permutation
// rebuild) with the replay-supplied sorted key; with_next from the row flags, index from
// matched_index; unmatched run k with id `id` sits right before matched row `id`, so row
// i lands at i + #runs with id <= i.  The run ids were checked strictly increasing by
// k_dec_sections, so a tile finds its runs by binary search and ranks rows with one scan.
__global__ void __launch_bounds__(256) k_dec_records(const DUnit* __restrict__ units, const int4* __restrict__ tiles,
                                                     const uint8_t* __restrict__ in, const int32_t* __restrict__ cinv,
                                                     const uint8_t* __restrict__ wnf, const uint64_t* __restrict__ uidd,
                                                     const int2* __restrict__ keys, int4* __restrict__ rec) {
  constexpr int TR = kRecTile, PER = TR / 256;
  __shared__ int32_t mk[TR + 1];
  __shared__ int32_t lds[4];
  const int4 T = tiles[blockIdx.x];  // {unit, tile, first and past-the-last run of the tile} (k_dec_fill_tiles)
  const DUnit u = units[T.x];
  const int32_t M = u.M;
  const int32_t i0 = T.y * TR;
  const int32_t n = max(0, min(TR, M - i0));
  const uint64_t* ids = uidd + u.wbase;
  for (int r = threadIdx.x; r <= TR; r += 256) mk[r] = 0;
  __syncthreads();
  const int32_t lo = T.z, hi = T.w;
  for (int32_t k = lo + threadIdx.x; k < hi; k += 256) {
    const int32_t id = (int32_t)ids[k];
    mk[id - i0] = 1;
    const int64_t at = u.rec_off + id + k;
    const int32_t cnt = (int32_t)ld_u64(in + u.ucnt_off + 8ll * k);
    rec[2 * at] = make_int4(cnt, 2, 0, 0);
    rec[2 * at + 1] = make_int4(0, 0, 0, u.set_id);
  }
  __syncthreads();
  // runs before row r (inclusive of a run with id == r): scan in thread-contiguous order,
  // then rows are written lane-contiguous so that each store instruction covers 2 KiB
  int32_t tot = 0;
#pragma unroll
  for (int q = 0; q < PER; q++) tot += mk[threadIdx.x * PER + q];
  int32_t all;
  int32_t run = block_exclusive_scan<256>(tot, 0, OpAdd(), lds, &all) + lo;
#pragma unroll
  for (int q = 0; q < PER; q++) {
    run += mk[threadIdx.x * PER + q];
    mk[threadIdx.x * PER + q] = run;  // each thread rewrites only its own entries
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < PER; q++) {
    const int32_t r = q * 256 + threadIdx.x;
    if (r >= n) break;
    const int32_t i = i0 + r;
    const int64_t at = u.rec_off + i + mk[r];
    const int2 k = keys[u.key_off + cinv[u.key_off + i]];
    const int32_t idx = (u.Mi > 0) ? (int32_t)ld_u64(in + u.mi_off + 8ll * i) : 0;  // Mi is M or 0 (rep files)
    rec[2 * at] = make_int4(1, 2, 1, k.x);
    rec[2 * at + 1] = make_int4(wnf[u.wbase + i], idx, k.y, u.set_id);
  }
}

// Round-trip check on the device: record i of encoder unit u's T-order range is input record
// rec_off[rank] + the stream position kept in its T-order record; after encode + decode of the
// same batch the unit's decoded records (dec_off[u] on) must be the fields the replay side can
// rebuild, in the same order: a matched event as {1, 2, 1, source, with_next as 0/1, index,
// clock, set}, and every maximal run of unmatched polls as ONE record {sum of the run's counts,
// 2, 0, 0, 0, 0, 0, set} (the encoder merges the polls before a matched event into one run).
// Input record i therefore lands at decoded index #(matched events and run starts before i);
// the thread of a run's first poll adds up the run.
__global__ void __launch_bounds__(256) k_verify_roundtrip(const Unit* __restrict__ units, const int64_t* __restrict__ dec_off,
                                                          const int64_t* __restrict__ rec_off,
                                                          const TRec* __restrict__ trec, const int4* __restrict__ rec_in,
                                                          const int4* __restrict__ rec_out,
                                                          unsigned long long* __restrict__ bad) {
  __shared__ int32_t lds[4];
  const Unit u = units[blockIdx.x];
  const int64_t rb = rec_off[u.rank], ob = dec_off[blockIdx.x];
  const int64_t n_out = dec_off[blockIdx.x + 1] - ob;
  auto in_rec = [&](int32_t i) { return rb + (int64_t)(trec[u.a + i].info & kInfoPos); };
  int32_t nbad = 0, carry = 0;
  for (int32_t i0 = 0; i0 < u.n; i0 += 256) {
    const int32_t i = i0 + threadIdx.x;
    const bool ok = i < u.n;
    int4 lo = make_int4(0, 0, 0, 0), hi = lo;
    bool m = false, emits = false;
    if (ok) {
      const int64_t g = in_rec(i);
      lo = rec_in[2 * g];
      hi = rec_in[2 * g + 1];
      m = lo.z == 1;
      emits = m || i == 0 || rec_in[2 * in_rec(i - 1)].z == 1;  // a matched event, or the first poll of a run
    }
    int32_t tot;
    const int32_t at = carry + block_exclusive_scan<256>(emits ? 1 : 0, 0, OpAdd(), lds, &tot);
    carry += tot;
    if (!emits) continue;
    if (at >= n_out) {
      nbad++;
      continue;
    }
    int4 wa, wb;
    if (m) {
      wa = make_int4(1, 2, 1, lo.w);
      wb = make_int4(hi.x != 0 ? 1 : 0, hi.y, hi.z, hi.w);
    } else {
      int32_t cnt = lo.x;
      for (int32_t k = i + 1; k < u.n; k++) {
        const int4 q = rec_in[2 * in_rec(k)];
        if (q.z == 1) break;
        cnt = (int32_t)((uint32_t)cnt + (uint32_t)q.x);  // (the encoder's sum wraps in 32 bits)
      }
      wa = make_int4(cnt, 2, 0, 0);
      wb = make_int4(0, 0, 0, hi.w);
    }
    const int4 a = rec_out[2 * (ob + at)], b = rec_out[2 * (ob + at) + 1];
    if (a.x != wa.x || a.y != wa.y || a.z != wa.z || a.w != wa.w || b.x != wb.x || b.y != wb.y || b.z != wb.z ||
        b.w != wb.w)
      nbad++;
  }
  if (threadIdx.x == 0 && carry != n_out) nbad++;  // (records the decode has and the input does not account for)
  nbad = wave_reduce(nbad, OpAdd());
  if (lane_id() == 0 && nbad) atomicAdd(bad, (unsigned long long)nbad);
}

}  // namespace cdcx

namespace cdcx {

// Host copy of the decoded tables (replay pipeline / table dumps): one block per unit packs
// the live prefixes of its M+1-strided scratch rows -- with_previous[W], unmatched ids[U],
// pair ids[P], pair delays[P] -- contiguously at pk_off[unit], so the D2H carries only
// what the tables hold.
__global__ __launch_bounds__(256) void k_dec_pack_tables(const DUnit* __restrict__ units,
                                                         const int64_t* __restrict__ pk_off,
                                                         const uint64_t* __restrict__ wpd,
                                                         const uint64_t* __restrict__ uidd,
                                                         const uint64_t* __restrict__ idd,
                                                         const uint64_t* __restrict__ dld,
                                                         uint64_t* __restrict__ pk) {
  const DUnit u = units[blockIdx.x];
  uint64_t* o = pk + pk_off[blockIdx.x];
  const int32_t U = u.Uc > 0 ? u.U : 0;
  for (int32_t i = threadIdx.x; i < u.W; i += blockDim.x) o[i] = wpd[u.wbase + i];
  o += u.W;
  for (int32_t i = threadIdx.x; i < U; i += blockDim.x) o[i] = uidd[u.wbase + i];
  o += U;
  for (int32_t i = threadIdx.x; i < u.P; i += blockDim.x) o[i] = idd[u.wbase + i];
  o += u.P;
  for (int32_t i = threadIdx.x; i < u.P; i += blockDim.x) o[i] = dld[u.wbase + i];
}

}  // namespace cdcx
