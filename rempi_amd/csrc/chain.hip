// chain.hip -- the CDC chain (rempi_clock_delta_compression.cpp:93-257, :465-551) computed
// segment-parallel on gfx950.
//
// Rule being reproduced (oracle/cdc_oracle.cpp ChainBuilder): node i = (row i, column c[i]);
// level(i) = 1 + max level of earlier nodes with a smaller column (exact LIS DP); its parent
// is, scanning the childless nodes ("leaves") in creation order, the level-(level(i)-1)
// ancestor of the first leaf whose such ancestor has a smaller column; a parent that was a
// leaf stops being one; when a node lands on the first untaken column, leaves left of it
// are dropped.  The chain is the parent path of the final node (M, M), whose parent is the
// earliest node of maximal level.
//
// Decomposition.  Cut the permutation at every closed prefix (max(c[0..r]) == r).  Every
// node after a cut sees every node before it as valid, so a segment's internal structure
// (relative levels, parents at relative level >= 2, leaf list) does not depend on earlier
// segments.  Only relative-level-1 nodes have a parent outside: the j-th such node of a
// segment takes the j-th max-level node of the previous segment ("Q", all still leaves),
// and once Q is used up it shares the parent of the relative-level-1 ancestor of the
// segment's first leaf.  Segments are therefore simulated independently (one lane each,
// state in registers) and stitched by k_chain_resolve.
//
// Per lane per event: k* from a register cache of the top TC patience-pile tops (the
// column of the latest node of each of the highest levels); the first leaf (register
// slots, creation order) whose level-k* ancestor has a smaller column wins; ancestors
// deeper than the leaf itself are reached through the parent array.  A leaf list longer
// than NL slots spills to global memory and that segment finishes on the exact slow path.
#include <hip/hip_runtime.h>

#include "cdcx_device.h"
#include "cdcx_kernels.h"

namespace cdcx {

// Segment ends: rows r with max(c[0..r]) == r.  One workgroup per unit.
__global__ void __launch_bounds__(256) k_cuts(Unit* __restrict__ units, const int32_t* __restrict__ cord,
                                              int32_t* __restrict__ segend) {
  __shared__ int32_t lds[4];
  Unit& u = units[blockIdx.x];
  const int64_t a = u.a;
  const int32_t M = u.M;
  int32_t cmax = -1, cn = 0;
  for (int32_t b = 0; b < M; b += 256) {
    const int32_t r = b + threadIdx.x;
    const bool valid = r < M;
    const int32_t v = valid ? cord[a + r] : -1;
    int32_t tmax;
    const int32_t ex = block_exclusive_scan<256>(v, -1, OpMax(), lds, &tmax);
    const int32_t inc = max(max(ex, cmax), v);
    const bool cut = valid && inc == r;
    int32_t tc;
    const int32_t pos = block_exclusive_scan<256>((int32_t)cut, 0, OpAdd(), lds, &tc);
    if (cut) segend[a + cn + pos] = r;
    cn += tc;
    cmax = max(cmax, tmax);
  }
  if (threadIdx.x == 0) u.nseg = cn;
}

__global__ void __launch_bounds__(256) k_seg_list(const Unit* __restrict__ units, const int32_t* __restrict__ segend,
                                                  Seg* __restrict__ segs) {
  const Unit u = units[blockIdx.x];
  for (int32_t k = threadIdx.x; k < u.nseg; k += 256) {
    const int32_t e = segend[u.a + k];
    const int32_t s = (k == 0) ? 0 : segend[u.a + k - 1] + 1;
    segs[u.seg0 + k] = Seg{(int32_t)blockIdx.x, k, s, e - s + 1, 0, 0, 0, 0};
  }
}

namespace {

constexpr int kTopCache = 8;

struct SegCtx {
  int64_t a;            // unit T-order base (node arrays are indexed a + row)
  int32_t s0, s1;       // rows [s0, s1)
  int32_t ord;
  int64_t lbase;        // global leaf-list base for the slow path
};

__device__ __forceinline__ int32_t climb(const int32_t* __restrict__ par, int64_t a, int32_t s, int32_t d) {
  for (; d > 0; d--) s = par[a + s];
  return s;
}

}  // namespace

template <int NL>
__global__ void __launch_bounds__(256) k_chain_seg(const Unit* __restrict__ units, Seg* __restrict__ segs, int32_t nsegs,
                                                   int32_t* __restrict__ queue, const int32_t* __restrict__ cord,
                                                   const int32_t* __restrict__ inv, int32_t* __restrict__ par,
                                                   int32_t* __restrict__ lvl, int32_t* __restrict__ exta,
                                                   int32_t* __restrict__ topg, int32_t* __restrict__ qn,
                                                   int32_t* __restrict__ leafg, const int64_t* __restrict__ w1,
                                                   uint32_t* err) {
  // Work distribution: block b owns the contiguous segments [b*nsegs/B, (b+1)*nsegs/B) and
  // its lanes take them one at a time from an LDS counter (no global atomics).
  __shared__ int32_t next_seg;
  const int32_t seg_lo = (int32_t)((int64_t)blockIdx.x * nsegs / gridDim.x);
  const int32_t seg_hi = (int32_t)((int64_t)(blockIdx.x + 1) * nsegs / gridDim.x);
  if (threadIdx.x == 0) next_seg = seg_lo;
  __syncthreads();
  // lane state
  int32_t si = -1;
  SegCtx S{0, 0, 0, 0, 0};
  int32_t i = 0, open = 0, nl = 0, lmax = 0, nrel1 = 0, qcnt = 0;
  bool slow = false;
  int32_t lid[NL], llv[NL], lcol[NL];
  int32_t topR[kTopCache];
#pragma unroll
  for (int s = 0; s < NL; s++) lid[s] = llv[s] = lcol[s] = 0;
#pragma unroll
  for (int j = 0; j < kTopCache; j++) topR[j] = 0;

  while (true) {
    if (i >= S.s1) {
      if (si >= 0) {
        segs[si].lmax = lmax;
        segs[si].qcount = qcnt;
      }
      si = atomicAdd(&next_seg, 1);
      if (si >= seg_hi) break;
      const Seg sg = segs[si];
      S.a = units[sg.unit].a;
      S.s0 = sg.start;
      S.s1 = sg.start + sg.len;
      S.ord = sg.ord;
      S.lbase = w1[sg.unit] + sg.start;
      i = S.s0;
      open = S.s0;
      nl = 0;
      lmax = 0;
      nrel1 = 0;
      qcnt = 0;
      slow = false;
      continue;
    }
    const int64_t a = S.a;
    const int32_t c = cord[a + i];

    // ---- k*: highest level holding a node with a smaller column -----------------------
    int32_t ks = -1;
#pragma unroll
    for (int j = 0; j < kTopCache; j++)
      if (ks < 0 && j < lmax && topR[j] < c) ks = lmax - j;
    if (ks < 0) {
      ks = 0;
      if (lmax > kTopCache) {  // binary search levels [1, lmax - kTopCache] of the global tops
        int32_t lo = 1, hi = lmax - kTopCache;  // largest k in [lo,hi] with top[k] < c
        while (lo <= hi) {
          const int32_t mid = (lo + hi) >> 1;
          if (topg[a + S.s0 + mid - 1] < c) { ks = mid; lo = mid + 1; } else hi = mid - 1;
        }
      }
    }

    // ---- parent ------------------------------------------------------------------------
    int32_t pnode = -1, pslot = -1;
    if (ks >= 1) {
      bool found = false;
      if (!slow) {
        // First slot (creation order) whose level-k* ancestor has a smaller column.  Slots
        // at level k* are checked in registers; a slot above k* needs a climb through the
        // parent array, done one slot at a time so the wave's lanes climb together.
        int32_t cursor = 0;
        while (true) {
          int32_t wa = NL, wb = NL;
#pragma unroll
          for (int s = NL - 1; s >= 0; s--) {
            if (s >= cursor && s < nl) {
              if (llv[s] == ks && lcol[s] < c) wa = s;
              if (llv[s] > ks) wb = s;
            }
          }
          if (wa < wb) {
            found = true;
            pslot = wa;
#pragma unroll
            for (int s = 0; s < NL; s++)
              if (s == wa) pnode = lid[s];
            break;
          }
          if (wb == NL) break;
          int32_t L = 0, d = 0;
#pragma unroll
          for (int s = 0; s < NL; s++)
            if (s == wb) { L = lid[s]; d = llv[s] - ks; }
          const int32_t anc = climb(par, a, L, d);
          if (cord[a + anc] < c) {
            found = true;
            pnode = anc;
            break;
          }
          cursor = wb + 1;
        }
      } else {
        for (int32_t q = 0; q < nl && !found; q++) {
          const int32_t L = leafg[S.lbase + q];
          const int32_t lv = lvl[a + L];
          if (lv < ks) continue;
          const int32_t anc = climb(par, a, L, lv - ks);
          if (cord[a + anc] < c) {
            found = true;
            pnode = anc;
            pslot = (anc == L) ? q : -1;
          }
        }
      }
      if (!found) raise_error(err, kErrCorrupt);  // cannot happen for a valid permutation
      par[a + i] = pnode;
    } else if (S.ord == 0) {
      par[a + i] = -1;  // first segment: level 1 hangs off the root
    } else {
      // Outside parent: resolved by k_chain_resolve from (ordinal, first leaf's anchor).
      par[a + i] = -2 - nrel1;
      int32_t anchor = -1;
      if (nl > 0) {
        const int32_t L = slow ? leafg[S.lbase] : lid[0];
        const int32_t lv = slow ? lvl[a + L] : llv[0];
        anchor = climb(par, a, L, lv - 1);
      }
      exta[a + i] = anchor;
      nrel1++;
    }

    // ---- node, tops, max-level list -----------------------------------------------------
    const int32_t k = ks + 1;
    lvl[a + i] = k;
    topg[a + S.s0 + ks] = c;
    if (k > lmax) {
#pragma unroll
      for (int j = kTopCache - 1; j > 0; j--) topR[j] = topR[j - 1];
      topR[0] = c;
      lmax = k;
      qcnt = 0;
    } else {
#pragma unroll
      for (int j = 0; j < kTopCache; j++)
        if (j == lmax - k) topR[j] = c;
    }
    if (k == lmax) qn[a + S.s0 + qcnt++] = i;

    // ---- leaf list: drop the adopted leaf, append the new node, sweep ---------------------
    if (!slow) {
      if (pslot >= 0) {
#pragma unroll
        for (int s = 0; s < NL - 1; s++)
          if (s >= pslot && s + 1 < nl) {
            lid[s] = lid[s + 1];
            llv[s] = llv[s + 1];
            lcol[s] = lcol[s + 1];
          }
        nl--;
        pslot = -1;  // done; the slow block below must not erase again
      }
      if (nl == NL) {  // spill and continue exactly on the slow path
#pragma unroll
        for (int s = 0; s < NL; s++) leafg[S.lbase + s] = lid[s];
        slow = true;
      } else {
#pragma unroll
        for (int s = 0; s < NL; s++)
          if (s == nl) {
            lid[s] = i;
            llv[s] = k;
            lcol[s] = c;
          }
        nl++;
      }
    }
    if (slow) {
      if (pslot >= 0) {
        for (int32_t q = pslot; q + 1 < nl; q++) leafg[S.lbase + q] = leafg[S.lbase + q + 1];
        nl--;
      }
      leafg[S.lbase + nl++] = i;
    }
    if (c == open) {
      if (!slow) {
        for (int rep = 0; rep < NL; rep++) {
          int d = -1;
#pragma unroll
          for (int s = NL - 1; s >= 0; s--)
            if (s < nl && lcol[s] < open) d = s;
          if (d < 0) break;
#pragma unroll
          for (int s = 0; s < NL - 1; s++)
            if (s >= d && s + 1 < nl) {
              lid[s] = lid[s + 1];
              llv[s] = llv[s + 1];
              lcol[s] = lcol[s + 1];
            }
          nl--;
        }
      } else {
        int32_t w = 0;
        for (int32_t q = 0; q < nl; q++) {
          const int32_t L = leafg[S.lbase + q];
          if (cord[a + L] >= open) leafg[S.lbase + w++] = L;
        }
        nl = w;
      }
    }
    while (open < S.s1 && inv[a + open] <= i) open++;
    i++;
  }
}

template __global__ void k_chain_seg<16>(const Unit*, Seg*, int32_t, int32_t*, const int32_t*, const int32_t*, int32_t*,
                                         int32_t*, int32_t*, int32_t*, int32_t*, int32_t*, const int64_t*, uint32_t*);

// Stitching.  From a max-level node of segment s, parents lead down to a relative-level-1
// node; its outside parent is Q[j] of segment s-1 where j is its ordinal, or, when j >= |Q|,
// that of its anchor (an earlier relative-level-1 node), repeatedly.
__device__ __forceinline__ int32_t seg_exit(const int32_t* __restrict__ par, const int32_t* __restrict__ exta,
                                            int64_t a, int32_t v, int32_t qprev, uint32_t* err) {
  int32_t p = par[a + v];
  while (p >= 0) {
    v = p;
    p = par[a + v];
  }
  int32_t j = -2 - p, guard = 0;
  while (j >= qprev) {
    v = exta[a + v];
    if (v < 0 || ++guard > (1 << 28)) { raise_error(err, kErrCorrupt); return 0; }
    j = -2 - par[a + v];
  }
  return j;
}

// Where the chain leaves segment s (ord > 0) for each of its max-level nodes.
__global__ void __launch_bounds__(256) k_chain_exits(const Unit* __restrict__ units, const Seg* __restrict__ segs,
                                                     int32_t nsegs, const int32_t* __restrict__ par,
                                                     const int32_t* __restrict__ exta, const int32_t* __restrict__ qn,
                                                     int32_t* __restrict__ qexit, uint32_t* err) {
  const int si = blockIdx.x * 256 + threadIdx.x;
  if (si >= nsegs) return;
  const Seg sg = segs[si];
  if (sg.ord == 0) return;
  const int64_t a = units[sg.unit].a;
  const int32_t qprev = segs[si - 1].qcount;
  for (int32_t j = 0; j < sg.qcount; j++) qexit[a + sg.start + j] = seg_exit(par, exta, a, qn[a + sg.start + j], qprev, err);
}

// Per unit: chain entry index of every segment, last to first; chain length.
__global__ void __launch_bounds__(64) k_chain_entries(Unit* __restrict__ units, int32_t n_units, Seg* __restrict__ segs,
                                                      const int32_t* __restrict__ qexit) {
  const int ui = blockIdx.x * 64 + threadIdx.x;
  if (ui >= n_units) return;
  Unit& u = units[ui];
  int32_t j = 0, K = 0;
  for (int32_t s = u.nseg - 1; s >= 0; s--) {
    Seg& sg = segs[u.seg0 + s];
    sg.entry = j;
    K += sg.lmax;
    if (s > 0) j = qexit[u.a + sg.start + j];
  }
  u.K = K;
  u.P = u.M - K;
}

// Mark the chain inside every segment: from its entry node down to relative level 1.
__global__ void __launch_bounds__(256) k_chain_mark(const Unit* __restrict__ units, const Seg* __restrict__ segs,
                                                    int32_t nsegs, const int32_t* __restrict__ par,
                                                    const int32_t* __restrict__ qn, uint8_t* __restrict__ chain) {
  const int si = blockIdx.x * 256 + threadIdx.x;
  if (si >= nsegs) return;
  const Seg sg = segs[si];
  const int64_t a = units[sg.unit].a;
  int32_t v = qn[a + sg.start + sg.entry];
  while (true) {
    chain[a + v] = 1;
    const int32_t p = par[a + v];
    if (p < 0) break;
    v = p;
  }
}

}  // namespace cdcx
