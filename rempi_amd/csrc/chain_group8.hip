// chain_group8.hip -- the segment chain simulation (chain.hip, chain_group.hip) with one
// segment per group of EIGHT lanes: eight segments per wave.
//
// The chain kernel is bound by vector-instruction issue, and a 16-lane group uses its lanes
// badly: the leaf list of the bench traces holds 5-6 entries on average (8 or fewer for 96 %
// of the events) although almost every segment reaches 10-14 at some point.  Here lane j of a
// group holds leaf slot j AND leaf slot 8 + j (two register sets, "A" and "B"): the B set is
// touched only in iterations in which some group of the wave has more than eight leaves
// (wave-uniform branches), so the common iteration costs about what a 16-lane iteration
// costs and advances twice as many segments.  Same rule, same outputs (par, exta, topg, qn,
// segs[].lmax/qcount) and the same hand-over to the next tier when a list outgrows its 16
// slots as k_chain_grp<16>.
//
// What keeps the instruction count down:
//  * one word per row: the column with the "open" flag in bit 31 (k_cuts), streamed through a
//    two-register window per lane that shifts down one lane per row (DPP);
//  * the eight groups of a wave slide their windows in the same iteration: a segment that
//    starts at wave phase t puts its first row at window slot t, so the flush of the parent
//    buffer and the window loads sit behind a scalar branch taken every eighth iteration;
//  * 32-bit byte offsets from the (scalar) array bases for every global access -- the host
//    launches this kernel only when the batch has fewer than 2^30 rows;
//  * group ballots as scalar compare masks (no select/compare round trip per ballot);
//  * ancestor climbs read the LDS ring directly; the global fallback for rows older than the
//    ring sits behind a branch;
//  * the single-word outputs are combined in LDS: the spilled tops (levels below the eight in
//    registers) live in a per-group ring of the last 32 spilled levels that is written to
//    topg one whole 128-byte line at a time, and never at all for levels that are still in
//    the ring when the segment ends; the max-level rows (qn) are kept in LDS and stored once
//    at the end of the segment.  One word at a time, these stores left partly written lines
//    in more groups than the L2 holds and went to memory several times per line.
//
// 8-lane groups on 16-lane DPP rows: a row shift leaks one value of the neighbouring group
// into lane 7 (row_shl) or lane 0 (row_shr) of a group; every use below either overwrites
// that lane or leaves it outside the live part of the list / window.  Broadcasts of a group's
// lane 0 are two bank-masked row_newbcast moves.
#include <hip/hip_runtime.h>

#include "cdcx_device.h"
#include "cdcx_kernels.h"

namespace cdcx {

namespace {
constexpr int G8 = 8;
// Rows of {par, column} per group in LDS.  Five blocks per CU hold their rings for the whole
// kernel, and the LDS they leave decides how many blocks of the other streams' kernels run beside
// them: with 64 rows (27.6 KB per block) this kernel and everything next to it ran a third slower.
// Climbs in near-sorted traces stay within 32 rows; older rows are read from memory.
constexpr int kRing8 = 32;
constexpr int kTopRing = 32;    // spilled tops per group in LDS: one 128-byte line of topg
constexpr int kQBuf = 8;        // max-level rows per group kept in LDS until the segment ends

using mask64 = unsigned long long;
// lane masks of a signed compare, straight from v_cmp (LLVM integer predicates)
__device__ __forceinline__ mask64 m_lt(int32_t x, int32_t y) { return __builtin_amdgcn_sicmp(x, y, 40); }
__device__ __forceinline__ mask64 m_gt(int32_t x, int32_t y) { return __builtin_amdgcn_sicmp(x, y, 38); }
__device__ __forceinline__ mask64 m_eq(int32_t x, int32_t y) { return __builtin_amdgcn_sicmp(x, y, 32); }
__device__ __forceinline__ mask64 m_ne(int32_t x, int32_t y) { return __builtin_amdgcn_sicmp(x, y, 33); }
__device__ __forceinline__ mask64 m_ge(int32_t x, int32_t y) { return __builtin_amdgcn_sicmp(x, y, 39); }
// the group's byte of a lane mask (sh = the group's first lane)
__device__ __forceinline__ uint32_t grp8(mask64 m, int sh) { return (uint32_t)(m >> sh) & 0xFFu; }

// value of the group's lane 0
__device__ __forceinline__ int32_t first8(int32_t v) {
  int32_t t = __builtin_amdgcn_update_dpp(0, v, 0x150, 0xf, 0x3, false);  // row_newbcast:0 -> lanes 0-7 of the row
  return __builtin_amdgcn_update_dpp(t, v, 0x158, 0xf, 0xC, false);       // row_newbcast:8 -> lanes 8-15
}
// lane j <- lane j+1 (the group's lane 7 receives the neighbouring group's lane 0, or 0: bound_ctrl, so
// that the instruction needs no copy of the old value)
__device__ __forceinline__ int32_t next8(int32_t v) { return __builtin_amdgcn_update_dpp(0, v, 0x101, 0xf, 0xf, true); }
// lane j <- lane j-1 (the group's lane 0 receives the neighbouring group's lane 7, or 0)
__device__ __forceinline__ int32_t prev8(int32_t v) { return __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true); }
__device__ __forceinline__ uint32_t below(int j) { return (1u << j) - 1u; }

// global accesses at a 32-bit byte offset from a wave-uniform base
__device__ __forceinline__ int32_t ldg(const int32_t* base, uint32_t boff) {
  return *reinterpret_cast<const int32_t*>(reinterpret_cast<const char*>(base) + boff);
}
__device__ __forceinline__ void stg(int32_t* base, uint32_t boff, int32_t v) {
  *reinterpret_cast<int32_t*>(reinterpret_cast<char*>(base) + boff) = v;
}
#ifdef CDCX_CHAIN_STATS
// Wave-level path counts (profiling build only): the first active lane of the wave counts.
__device__ unsigned long long g8_stats[24];
#define G8_STAT(n)                                                                               \
  do {                                                                                           \
    if ((int)(threadIdx.x & 63) == __ffsll((long long)__builtin_amdgcn_ballot_w64(true)) - 1) st[n]++; \
  } while (0)
#else
#define G8_STAT(n) do { } while (0)
#endif
}  // namespace

#ifdef CDCX_CHAIN_STATS
extern "C" int cdcx_debug_g8_stats(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g8_stats), sizeof(g8_stats)) != hipSuccess) return 1;
  if (reset) {
    unsigned long long z[24] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g8_stats), z, sizeof(z)) != hipSuccess) return 1;
  }
  return 0;
}
#endif

__global__ void __launch_bounds__(256) k_chain_grp8(const Unit* __restrict__ units, Seg* __restrict__ segs,
                                                    const int32_t* __restrict__ list, const int32_t* __restrict__ nlist_p,
                                                    const int32_t* __restrict__ cord, const int32_t* __restrict__ opn,
                                                    int32_t* __restrict__ par, int32_t* __restrict__ exta,
                                                    int32_t* __restrict__ topg, int32_t* __restrict__ qn,
                                                    int32_t* __restrict__ ovf, int32_t* __restrict__ novf, int32_t long_len,
                                                    uint32_t* err) {
  constexpr int G = G8;
  constexpr int kGroups = 256 / G;
  constexpr int R = kRing8;
  __shared__ int32_t next_j;
  __shared__ int2 ring_all[kGroups][R];          // {par, column} of row r at [r % R]
  __shared__ int32_t comp_all[kGroups][3 * 16];  // sweep compaction of a list that uses the B slots
  __shared__ int32_t tring_all[kGroups][kTopRing];  // spilled top of level e + 1 at [(tq + e) % 32]
  __shared__ int32_t qbuf_all[kGroups][kQBuf];
  int2* ring = ring_all[threadIdx.x / G];
  int32_t* comp = comp_all[threadIdx.x / G];
  int32_t* tring = tring_all[threadIdx.x / G];
  int32_t* qbuf = qbuf_all[threadIdx.x / G];
  if (threadIdx.x == 0) next_j = 0;
  __syncthreads();

  const int j = threadIdx.x & 7;
  const int sh = threadIdx.x & 56;     // the group's first lane in the wave
  const int32_t bp4 = sh << 2;         // its ds_bpermute / ds_permute address
  const int32_t nlist = *nlist_p;
  // group-uniform state.  ab / tb: byte offsets of the unit's row 0 / the segment's row 0.
  int32_t si = -1, s0 = 0, s1 = 0, ord = 0;
  uint32_t ab = 0, tb = 0;
  int32_t tq = 0;  // word index of the segment's topg row 0 (tb / 4): lines of topg are 32-word aligned in it
  int32_t i = 0, nl = 0, lmax = 0, nrel1 = 0, qcnt = 0;
  bool islong = false;
  // lane state: leaf slots j (A) and 8 + j (B), top of level lmax - j, the row window (row
  // i + j in cw0 while it lies in the current eight-row frame, the next frame in cw1), the
  // frame's parents (row rj = frame start + j)
  int32_t lid = 0, llv = 0, lcol = 0, lidB = 0, llvB = 0, lcolB = 0;
  int32_t top = 0, cw0 = 0, cw1 = 0, pval = 0, rj = j;
  // wave-uniform phase: every group's row i sits at slot t of its frame
  int t = 0;
#ifdef CDCX_CHAIN_STATS
  unsigned long long st[24] = {};
#endif

  auto ring_par = [&](int32_t x) -> int32_t {  // parent of row x < i of this segment
    int32_t p = ring[x & (R - 1)].x;
    asm volatile("" : "+v"(p));  // keeps the LDS read an LDS read (no flat load of a selected address)
#ifdef CDCX_CHAIN_STATS
    if (x < i - R) atomicAdd(&g8_stats[22], 1ull);
    if (x < i - 32) atomicAdd(&g8_stats[23], 1ull);
    if (x < i - 16) atomicAdd(&g8_stats[19], 1ull);
#endif
    if (x < i - R) p = ldg(par, ab + 4u * (uint32_t)x);
    return p;
  };
  auto ring_col = [&](int32_t x) -> int32_t {
    int32_t q = ring[x & (R - 1)].y;
    asm volatile("" : "+v"(q));
    if (x < i - R) q = ldg(cord, ab + 4u * (uint32_t)x);
    return q;
  };

  while (true) {
    G8_STAT(0);
    if (t == G) {  // every group at once: store the frame's parents, slide the windows
      t = 0;
      if (rj >= s0) stg(par, ab + 4u * (uint32_t)rj, pval);  // (rows before s0: the previous segment's, stored there)
      rj += G;
      cw0 = cw1;
      cw1 = (rj + G < s1) ? ldg(opn, ab + 4u * (uint32_t)rj + 4u * G) : 0;
      // The kernel ends when its longest segments end, and they share their SIMD with other
      // waves all the way: a wave that runs one of them issues ahead of the others.
      if (__builtin_amdgcn_ballot_w64(islong) != 0)
        __builtin_amdgcn_s_setprio(3);
      else
        __builtin_amdgcn_s_setprio(0);
    }
    if (i >= s1) {
      G8_STAT(1);
      if (si >= 0) {
        if (j < t && rj >= s0) stg(par, ab + 4u * (uint32_t)rj, pval);
        if (j < min(qcnt, kQBuf)) stg(qn, tb + 4u * (uint32_t)j, qbuf[j]);
        if (j == 0) {
          segs[si].lmax = lmax;
          segs[si].qcount = qcnt;
        }
      }
      int32_t k = 0;
      if (j == 0) k = atomicAdd(&next_j, 1);
      k = first8(k);
      const int64_t kk = (int64_t)blockIdx.x + (int64_t)gridDim.x * k;
      if (kk >= nlist) break;
      G8_STAT(20);
      si = list[kk];
      const Seg sg = segs[si];
      ab = (uint32_t)units[sg.unit].a << 2;
      s0 = sg.start;
      s1 = sg.start + sg.len;
      ord = sg.ord;
      tb = ab + 4u * (uint32_t)s0;
      tq = (int32_t)(tb >> 2);
      i = s0;
      rj = s0 - t + j;
      nl = lmax = nrel1 = qcnt = 0;
      islong = sg.len >= long_len;
      cw0 = (j < G - t && s0 + j < s1) ? ldg(opn, tb + 4u * j) : 0;
      cw1 = (rj + G < s1) ? ldg(opn, ab + 4u * (uint32_t)(rj + G)) : 0;
    }
    const int32_t cv = first8(cw0);  // row i: column, bit 31 = first column not taken by rows < i
    cw0 = next8(cw0);
    const int32_t c = cv & 0x7fffffff;
    // does any group of this wave use its B slots in this iteration?
    const bool useB = m_gt(nl, G) != 0;
    G8_STAT(2);
    if (useB) G8_STAT(3);
#ifdef CDCX_CHAIN_STATS
    st[21] += __popcll(__builtin_amdgcn_ballot_w64(true));
#endif

    // ---- k*: highest level whose top column is smaller than c ---------------------------
    const uint32_t tm = grp8(m_lt(j, lmax) & m_lt(top, c), sh);
    int32_t ks = tm ? lmax - (__ffs(tm) - 1) : 0;
    if (tm == 0 && lmax > G) {  // below the register tops: binary search the spilled levels
      int32_t lo = 1, hi = lmax - G;
      G8_STAT(4);
      while (lo <= hi) {
        G8_STAT(5);
        const int32_t mid = (lo + hi) >> 1;
        // level mid = spill index mid - 1; the last kTopRing spilled levels are in the ring
        int32_t tv = tring[(tq + mid - 1) & (kTopRing - 1)];
        asm volatile("" : "+v"(tv));
        if (mid - 1 < lmax - G - kTopRing) tv = ldg(topg, tb + 4u * (uint32_t)mid - 4u);
        if (tv < c) {
          ks = mid;
          lo = mid + 1;
        } else {
          hi = mid - 1;
        }
      }
    }

    // ---- parent --------------------------------------------------------------------------
    // Branches below are on wave-level masks (scalar branches); what differs between the
    // groups of the wave is predicated, so no group's path leaves copies at a join.
    int32_t pv;
    uint32_t pslot;  // the adopted leaf's slot, 16 = none
    {
      const mask64 has = m_gt(ks, 0);  // groups with a level below the new node
      const mask64 jn = m_lt(j, nl) & has;
      uint32_t eq = grp8(jn & m_eq(llv, ks) & m_lt(lcol, c), sh);
      uint32_t gt = grp8(jn & m_gt(llv, ks), sh);
      if (useB) {
        const mask64 jnB = m_lt(j + G, nl) & has;
        eq |= grp8(jnB & m_eq(llvB, ks) & m_lt(lcolB, c), sh) << G;
        gt |= grp8(jnB & m_gt(llvB, ks), sh) << G;
      }
      const uint32_t wa = __builtin_ctz(eq | (1u << (2 * G)));  // first eligible level-k* leaf, 16 = none
      const uint32_t need = gt & below(wa);
      uint32_t win = wa, ok = 0;
      int32_t x = lid, xB = lidB;
      if (m_ne((int32_t)need, 0) != 0) {
        G8_STAT(7);
        // every slot before wa holding a deeper leaf climbs to its level-k* ancestor at once
        const bool mine = (need >> j) & 1u;
        int32_t col = 0x7fffffff;
        if (mine) {
#pragma unroll 1
          for (int32_t d = llv - ks; d > 0; d--) {
            G8_STAT(8);
            x = ring_par(x);
          }
          col = ring_col(x);
        }
        ok = grp8(m_lt(col, c), sh);
        if (useB) {
          const bool mineB = (need >> (j + G)) & 1u;
          int32_t colB = 0x7fffffff;
          if (mineB) {
#pragma unroll 1
            for (int32_t d = llvB - ks; d > 0; d--) xB = ring_par(xB);
            colB = ring_col(xB);
          }
          ok |= grp8(m_lt(colB, c), sh) << G;
        }
        win = ok ? (uint32_t)__ffs(ok) - 1u : wa;
      }
      const bool interior = ok != 0;  // the parent is an ancestor found by a climb, not a leaf
      if ((m_ge((int32_t)win, 2 * G) & has) != 0) {
        if (win >= 2 * G && ks > 0) raise_error(err, kErrCorrupt);  // cannot happen for a valid permutation
      }
      // the parent: slot win's ancestor (interior) or slot win's leaf itself, which is adopted
      const int32_t ad = bp4 + ((win & 7) << 2);
      pv = __builtin_amdgcn_ds_bpermute(ad, interior ? x : lid);
      if (useB) {
        const int32_t pB = __builtin_amdgcn_ds_bpermute(ad, interior ? xB : lidB);
        pv = win < G ? pv : pB;
      }
      pslot = interior ? 2u * G : min(win, 2u * G);
      if (m_lt(ks, 1) != 0) {  // some group's node is on level 1
        const bool none = ks < 1, outside = none && ord != 0;
        // first segment: level 1 hangs off the root; later segments: outside parent, resolved
        // at stitching from (ordinal, first leaf) -- chain.hip
        pv = none ? (ord == 0 ? -1 : -2 - nrel1) : pv;
        if (__builtin_amdgcn_ballot_w64(outside) != 0) {
          G8_STAT(11);
          const int32_t f = first8(lid);
          if (outside && j == 0) stg(exta, ab + 4u * (uint32_t)i, nl > 0 ? f : -1);
        }
        nrel1 += outside ? 1 : 0;
      }
    }
    pval = (j == t) ? pv : pval;
    if (j == 0) ring[i & (R - 1)] = make_int2(pv, c);

    // ---- tops ------------------------------------------------------------------------------
    const int32_t k = ks + 1;
    const bool grow = k > lmax;
    if (grow && lmax >= G) G8_STAT(12);
    if (!grow && lmax - k >= G) G8_STAT(13);
    if (grow && lmax >= G) {
      // spill index e = lmax - G (level e + 1) leaves the registers: into the ring, and the
      // line of topg that it completes goes to memory whole (words before the segment's
      // first belong to another segment's spill area and are left alone)
      const int32_t e = lmax - G;
      const int32_t w = (tq + e) & (kTopRing - 1);
      if (j == G - 1) tring[w] = top;
      if (w == kTopRing - 1) {
#pragma unroll
        for (int q = 0; q < kTopRing / G; q++) {
          const int32_t z = q * G + j;  // word of the line
          const int32_t ez = e - (kTopRing - 1) + z;
          const int32_t v = tring[z];
          if (ez >= 0) stg(topg, tb + 4u * (uint32_t)ez, v);
        }
      }
    }
    if (!grow && lmax - k >= G && j == 0) {
      // a spilled level gets a new top: in the ring while it is among the last kTopRing
      // spilled, and in memory when its line has been written already
      const int32_t e = k - 1, n = lmax - G;  // n spilled levels so far
      if (e >= n - kTopRing) tring[(tq + e) & (kTopRing - 1)] = c;
      if (e < ((tq + n) & ~(kTopRing - 1)) - tq) stg(topg, tb + 4u * (uint32_t)e, c);
    }
    const int32_t tshift = prev8(top);
    top = grow ? ((j == 0) ? c : tshift) : ((j == lmax - k) ? c : top);
    qcnt = grow ? 0 : qcnt;
    lmax = grow ? k : lmax;
    if (k == lmax) G8_STAT(14);
    if (k == lmax && j == 0) {
      if (qcnt < kQBuf) qbuf[qcnt] = i;
      else stg(qn, tb + 4u * (uint32_t)qcnt, i);
    }
    qcnt += (k == lmax) ? 1 : 0;

    // ---- leaves: drop the adopted one, sweep, append the new node --------------------------
    {
      int32_t nid = next8(lid), nlv = next8(llv), ncol = next8(lcol);
      if (useB) {
        // slot 7 takes slot 8; the B slots shift down from the dropped slot on
        const int32_t bid = first8(lidB), blv = first8(llvB), bcol = first8(lcolB);
        if (j == G - 1) {
          nid = bid;
          nlv = blv;
          ncol = bcol;
        }
        const int32_t nidB = next8(lidB), nlvB = next8(llvB), ncolB = next8(lcolB);
        const bool dropB = j + G >= (int32_t)pslot;
        lidB = dropB ? nidB : lidB;
        llvB = dropB ? nlvB : llvB;
        lcolB = dropB ? ncolB : lcolB;
      }
      const bool drop = j >= (int32_t)pslot;
      lid = drop ? nid : lid;
      llv = drop ? nlv : llv;
      lcol = drop ? ncol : lcol;
      nl -= (pslot < 2 * G) ? 1 : 0;
    }
    // (the sweep comes before the append: the new node, on the open column itself, is never swept)
    {
      const mask64 sw = m_lt(cv, 0);  // groups whose row is on its first untaken column
      if (sw != 0) {
        G8_STAT(15);
        uint32_t dead = grp8(sw & m_lt(j, nl) & m_lt(lcol, c), sh);
        if (!useB) {
          if (m_ne((int32_t)dead, 0) != 0) {
            G8_STAT(16);
            // (a group without dead leaves permutes its live slots onto themselves)
            const bool alive = j < nl && !((dead >> j) & 1u);
            const int32_t dst = alive ? j - __popc(dead & below(j)) : G - 1;
            const int32_t ad = bp4 + (dst << 2);
            lid = __builtin_amdgcn_ds_permute(ad, lid);
            llv = __builtin_amdgcn_ds_permute(ad, llv);
            lcol = __builtin_amdgcn_ds_permute(ad, lcol);
            nl -= __popc(dead);
          }
        } else {
          dead |= grp8(sw & m_lt(j + G, nl) & m_lt(lcolB, c), sh) << G;
          if (m_ne((int32_t)dead, 0) != 0) {
            G8_STAT(17);
            // compaction through LDS: slot s (alive) lands at s - #dead below it
            const bool aliveA = j < nl && !((dead >> j) & 1u), aliveB = j + G < nl && !((dead >> (j + G)) & 1u);
            if (aliveA) {
              const int32_t d = j - __popc(dead & below(j));
              comp[d] = lid;
              comp[16 + d] = llv;
              comp[32 + d] = lcol;
            }
            if (aliveB) {
              const int32_t d = j + G - __popc(dead & below(j + G));
              comp[d] = lidB;
              comp[16 + d] = llvB;
              comp[32 + d] = lcolB;
            }
            __builtin_amdgcn_wave_barrier();
            lid = comp[j];
            llv = comp[16 + j];
            lcol = comp[32 + j];
            lidB = comp[G + j];
            llvB = comp[16 + G + j];
            lcolB = comp[32 + G + j];
            __builtin_amdgcn_wave_barrier();
            nl -= __popc(dead);
          }
        }
      }
    }
    if (m_ge(nl, G) != 0) {  // some group's list fills its A slots: the append goes to a B slot
      const bool full = nl == 2 * G;
      if (__builtin_amdgcn_ballot_w64(full) != 0) {  // leaf list outgrows the group: hand the segment to the next tier
        G8_STAT(18);
        if (full && j == 0) ovf[atomicAdd(novf, 1)] = si;
        si = full ? -1 : si;
        s1 = full ? i + 1 : s1;  // the rest of this iteration runs on junk state and ends the segment
        nl = full ? 0 : nl;
      }
      const bool ap = j + G == nl;
      lidB = ap ? i : lidB;
      llvB = ap ? k : llvB;
      lcolB = ap ? c : lcolB;
    }
    {
      const bool ap = j == nl;
      lid = ap ? i : lid;
      llv = ap ? k : llv;
      lcol = ap ? c : lcol;
    }
    nl++;
    i++;
    t++;
  }
#ifdef CDCX_CHAIN_STATS
  for (int q = 0; q < 24; q++)
    if (st[q]) atomicAdd(&g8_stats[q], st[q]);
#endif
}

}  // namespace cdcx
