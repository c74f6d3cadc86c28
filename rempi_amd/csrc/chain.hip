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

// Segment ends and the "open" flag of every row, one workgroup per unit, in one pass over inv
// (inv[k] = row that takes column k).  With pm[k] = max(inv[0..k]):
//  * the prefix of rows 0..k is closed (holds exactly the columns 0..k) iff pm[k] == k -- the
//    same cuts as max(c[0..r]) == r;
//  * row i = inv[k] sits on the first column not taken by rows < i exactly when every smaller
//    column belongs to an earlier row, inv[k] > pm[k-1]: that is what the chain rule tests when
//    it compares a new node's column with current_column_of_start_it
//    (rempi_clock_delta_compression.cpp:252, :303-316).
// opn[i] = column of row i, with bit 31 set when the row is open: the one word per row the
// chain kernels stream.
__global__ void __launch_bounds__(256) k_cuts(Unit* __restrict__ units, const int32_t* __restrict__ inv,
                                              int32_t* __restrict__ segend, int32_t* __restrict__ opn) {
  __shared__ int32_t lds[4];
  Unit& u = units[blockIdx.x];
  if (u.wfail != 0) return;  // not ranked yet (k_window_rank), or already done
  const int64_t a = u.a;
  const int32_t M = u.M;
  int32_t cmax = -1, cn = 0;
  // 4 columns per thread per round; the next round's rows are loaded during this one
  int32_t vn[4];
  auto load = [&](int32_t r0) {
#pragma unroll
    for (int q = 0; q < 4; q++) vn[q] = (r0 + q < M) ? inv[a + r0 + q] : -1;
  };
  load(4 * threadIdx.x);
  for (int32_t b = 0; b < M; b += 1024) {
    const int32_t r0 = b + 4 * threadIdx.x;
    int32_t v[4], lm = -1;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      v[q] = vn[q];
      lm = max(lm, v[q]);
    }
    load(r0 + 1024);
    int32_t tmax;
    int32_t run = max(block_exclusive_scan<256>(lm, -1, OpMax(), lds, &tmax), cmax);
    bool cut[4];
    int32_t nc = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      if (r0 + q < M) opn[a + v[q]] = (r0 + q) | (v[q] > run ? INT32_MIN : 0);
      run = max(run, v[q]);
      cut[q] = r0 + q < M && run == r0 + q;
      nc += cut[q] ? 1 : 0;
    }
    int32_t tc;
    int32_t pos = cn + block_exclusive_scan<256>(nc, 0, OpAdd(), lds, &tc);
#pragma unroll
    for (int q = 0; q < 4; q++)
      if (cut[q]) segend[a + pos++] = r0 + q;
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

// Longest-first order of the segments (counting sort on the length, descending; lengths
// past kLenBins share the first bin): blocks take strided positions of this order so every
// block gets a similar amount of work, and a wave's lanes run segments of similar length.
// Counts are aggregated per block in LDS, so the global atomics are one per (block,
// length present in the block).
constexpr int kLenBins = 4096;
__device__ __forceinline__ int len_bin(int32_t len) { return kLenBins - 1 - min(len, kLenBins - 1); }

__global__ void __launch_bounds__(256) k_seg_hist(const Seg* __restrict__ segs, int32_t nsegs, int32_t* __restrict__ hist) {
  latency_kernel();
  __shared__ int32_t h[kLenBins];
  for (int q = threadIdx.x; q < kLenBins; q += 256) h[q] = 0;
  __syncthreads();
  for (int i = blockIdx.x * 1024 + threadIdx.x; i < min(nsegs, (int)(blockIdx.x + 1) * 1024); i += 256)
    atomicAdd(&h[len_bin(segs[i].len)], 1);
  __syncthreads();
  for (int q = threadIdx.x; q < kLenBins; q += 256)
    if (h[q]) atomicAdd(&hist[q], h[q]);
}

__global__ void __launch_bounds__(256) k_seg_bins(int32_t* __restrict__ hist) {
  latency_kernel();
  __shared__ int32_t lds[4];
  int32_t run = 0;
  for (int b = 0; b < kLenBins; b += 256) {
    const int32_t v = hist[b + threadIdx.x];
    int32_t tot;
    const int32_t ex = block_exclusive_scan<256>(v, 0, OpAdd(), lds, &tot);
    hist[b + threadIdx.x] = run + ex;
    run += tot;
  }
}

__global__ void __launch_bounds__(256) k_seg_order(const Seg* __restrict__ segs, int32_t nsegs, int32_t* __restrict__ hist,
                                                   int32_t* __restrict__ order) {
  latency_kernel();
  __shared__ int32_t h[kLenBins];
  for (int q = threadIdx.x; q < kLenBins; q += 256) h[q] = 0;
  __syncthreads();
  const int i0 = blockIdx.x * 1024;
  int bin[4], rk[4];
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int i = i0 + q * 256 + threadIdx.x;
    bin[q] = 0;
    rk[q] = 0;
    if (i < nsegs) {
      bin[q] = len_bin(segs[i].len);
      rk[q] = atomicAdd(&h[bin[q]], 1);
    }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < kLenBins; q += 256)
    if (h[q]) h[q] = atomicAdd(&hist[q], h[q]);
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int i = i0 + q * 256 + threadIdx.x;
    if (i < nsegs) order[h[bin[q]] + rk[q]] = i;
  }
}

namespace {

constexpr int kTopCache = 8;

__device__ __forceinline__ int32_t climb(const int32_t* __restrict__ par, int64_t a, int32_t s, int32_t d) {
  for (; d > 0; d--) s = par[a + s];
  return s;
}

// 4-wide cached reader of one lane's int32 stream (16-byte aligned groups).
struct Stream4 {
  int64_t base = -1;
  int4 v;
  __device__ __forceinline__ int32_t get(const int32_t* __restrict__ p, int64_t idx) {
    const int64_t g = idx & ~(int64_t)3;
    if (g != base) {
      v = *reinterpret_cast<const int4*>(p + g);
      base = g;
    }
    const int k = (int)(idx & 3);
    return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
  }
};

}  // namespace

template <int NL>
__global__ void __launch_bounds__(256) k_chain_seg(const Unit* __restrict__ units, Seg* __restrict__ segs,
                                                   const int32_t* __restrict__ nsegs_p,
                                                   const int32_t* __restrict__ order, const int32_t* __restrict__ cord,
                                                   const int32_t* __restrict__ opn, int32_t* __restrict__ par,
                                                   int32_t* __restrict__ exta, int32_t* __restrict__ topg,
                                                   int32_t* __restrict__ qn, int2* __restrict__ leafg,
                                                   const int64_t* __restrict__ w1, uint32_t* err,
                                                   unsigned long long* __restrict__ stats) {
  // stats (diagnostics, normally null): events, slow events, winner iterations, climb
  // steps, k* searches, spills, open-advance steps, max leaves
  unsigned long long st_ev = 0, st_slow = 0, st_win = 0, st_climb = 0, st_ks = 0, st_spill = 0, st_open = 0;
  int32_t st_maxnl = 0;
  // Block b runs positions b, b+B, b+2B, ... of the longest-first order; its lanes take them
  // one at a time from an LDS counter.
  __shared__ int32_t next_j;
  if (threadIdx.x == 0) next_j = 0;
  __syncthreads();
  const int32_t nsegs = *nsegs_p;  // (a count left on the device by the tier before: the host does not wait for it)
  int32_t si = -1;
  int64_t a = 0, lbase = 0;
  int32_t s0 = 0, s1 = 0, ord = 0;
  int32_t i = 0, open = 0, nl = 0, lmax = 0, nrel1 = 0, qcnt = 0;
  bool slow = false;
  int32_t lid[NL], llv[NL], lcol[NL];
  int32_t topR[kTopCache];  // topR[j] = column of the latest node at level lmax - j
#pragma unroll
  for (int s = 0; s < NL; s++) lid[s] = llv[s] = lcol[s] = 0;
#pragma unroll
  for (int j = 0; j < kTopCache; j++) topR[j] = 0;
  Stream4 cs, is;

  while (true) {
    if (i >= s1) {
      if (si >= 0) {
        segs[si].lmax = lmax;
        segs[si].qcount = qcnt;
      }
      const int64_t k = (int64_t)blockIdx.x + (int64_t)gridDim.x * atomicAdd(&next_j, 1);
      if (k >= nsegs) {
        if (stats) {
          atomicAdd(&stats[0], st_ev);
          atomicAdd(&stats[1], st_slow);
          atomicAdd(&stats[2], st_win);
          atomicAdd(&stats[3], st_climb);
          atomicAdd(&stats[4], st_ks);
          atomicAdd(&stats[5], st_spill);
          atomicAdd(&stats[6], st_open);
          atomicMax(&stats[7], (unsigned long long)st_maxnl);
        }
        break;
      }
      si = order[k];
      const Seg sg = segs[si];
      a = units[sg.unit].a;
      s0 = sg.start;
      s1 = sg.start + sg.len;
      ord = sg.ord;
      lbase = w1[sg.unit] + sg.start;
      i = s0;
      open = s0;
      nl = lmax = nrel1 = qcnt = 0;
      slow = false;
      continue;
    }
    const int32_t c = cs.get(cord, a + i);
    open = is.get(opn, a + i) < 0 ? c : -1;  // c when it is the first column not taken by rows < i (k_cuts)
    if (stats) {
      st_ev++;
      st_slow += slow;
      st_maxnl = max(st_maxnl, nl);
    }

    // ---- k*: highest level holding a node with a smaller column -----------------------
    int32_t ks = -1;
#pragma unroll
    for (int j = 0; j < kTopCache; j++)
      if (ks < 0 && j < lmax && topR[j] < c) ks = lmax - j;
    if (ks < 0) {
      ks = 0;
      if (stats && lmax > kTopCache) st_ks++;
      if (lmax > kTopCache) {  // binary search the spilled tops of levels [1, lmax - kTopCache]
        int32_t lo = 1, hi = lmax - kTopCache;
        while (lo <= hi) {
          const int32_t mid = (lo + hi) >> 1;
          if (topg[a + s0 + mid - 1] < c) { ks = mid; lo = mid + 1; } else hi = mid - 1;
        }
      }
    }

    // ---- parent ------------------------------------------------------------------------
    int32_t pnode = -1, pslot = -1;
    if (ks >= 1) {
      bool found = false;
      if (!slow) {
        // First slot (creation order) whose level-k* ancestor has a smaller column; slots at
        // level k* are decided in registers, a slot above k* needs one climb (one at a time,
        // so the wave's lanes climb together).
        int32_t cursor = 0;
        while (true) {
          if (stats) st_win++;
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
          if (stats) st_climb += d;
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
          const int2 L = leafg[lbase + q];
          if (L.y < ks) continue;
          const int32_t anc = climb(par, a, L.x, L.y - ks);
          if (cord[a + anc] < c) {
            found = true;
            pnode = anc;
            pslot = (anc == L.x) ? q : -1;
          }
        }
      }
      if (!found) raise_error(err, kErrCorrupt);  // cannot happen for a valid permutation
      par[a + i] = pnode;
    } else if (ord == 0) {
      par[a + i] = -1;  // first segment: level 1 hangs off the root
    } else {
      // Outside parent: resolved at stitching from (ordinal, anchor of the first leaf).
      par[a + i] = -2 - nrel1;
      // the first leaf; k_chain_exits climbs from it to its relative-level-1 ancestor
      exta[a + i] = nl > 0 ? (slow ? leafg[lbase].x : lid[0]) : -1;
      nrel1++;
    }

    // ---- tops (registers; spill only levels that leave the cache) and max-level list ----
    const int32_t k = ks + 1;
    if (k > lmax) {
      if (lmax - (kTopCache - 1) >= 1) topg[a + s0 + (lmax - (kTopCache - 1)) - 1] = topR[kTopCache - 1];
#pragma unroll
      for (int j = kTopCache - 1; j > 0; j--) topR[j] = topR[j - 1];
      topR[0] = c;
      lmax = k;
      qcnt = 0;
    } else if (lmax - k < kTopCache) {
#pragma unroll
      for (int j = 0; j < kTopCache; j++)
        if (j == lmax - k) topR[j] = c;
    } else {
      topg[a + s0 + k - 1] = c;
    }
    if (k == lmax) qn[a + s0 + qcnt++] = i;

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
        pslot = -1;
      }
      if (nl == NL) {  // spill and continue exactly on the slow path
#pragma unroll
        for (int s = 0; s < NL; s++) leafg[lbase + s] = make_int2(lid[s], llv[s]);
        slow = true;
        if (stats) st_spill++;
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
        for (int32_t q = pslot; q + 1 < nl; q++) leafg[lbase + q] = leafg[lbase + q + 1];
        nl--;
      }
      leafg[lbase + nl++] = make_int2(i, k);
    }
    if (c == open) {
      if (!slow) {
        uint32_t dead = 0;
#pragma unroll
        for (int s = 0; s < NL; s++)
          if (s < nl && lcol[s] < open) dead |= 1u << s;
        while (dead) {
          const int d = __ffs(dead) - 1;
#pragma unroll
          for (int s = 0; s < NL - 1; s++)
            if (s >= d && s + 1 < nl) {
              lid[s] = lid[s + 1];
              llv[s] = llv[s + 1];
              lcol[s] = lcol[s + 1];
            }
          nl--;
          dead = (dead & ~(1u << d));
          dead = (dead & ((1u << d) - 1)) | ((dead >> 1) & ~((1u << d) - 1));
        }
      } else {
        int32_t w = 0;
        for (int32_t q = 0; q < nl; q++) {
          const int2 L = leafg[lbase + q];
          if (cord[a + L.x] >= open) leafg[lbase + w++] = L;
        }
        nl = w;
      }
    }
    i++;
  }
}

template __global__ void k_chain_seg<16>(const Unit*, Seg*, const int32_t*, const int32_t*, const int32_t*, const int32_t*,
                                         int32_t*, int32_t*, int32_t*, int32_t*, int2*, const int64_t*, uint32_t*,
                                         unsigned long long*);

// Stitching.  From a max-level node of segment s, parents lead down to a relative-level-1
// node; its outside parent is Q[j] of segment s-1 where j is its ordinal, or, when j >= |Q|,
// that of its anchor -- the relative-level-1 ancestor of the segment's first leaf when the
// node was created (exta holds that leaf) -- repeatedly.
// Where the chain leaves segment s (ord > 0) for each of its max-level nodes: one wave per
// segment, grid-stride.  Every step of the walk (a node's parent, or a relative-level-1 node's
// anchor) leads to a lower row, so the walk is one sweep over the segment's rows from the top,
// 64 rows (a chunk) at a time and four chunks per memory round trip; a single thread doing it
// load by load pays a round trip per step, 250 steps for the average segment of a dense
// table.  In a chunk each lane holds the next step of its row; pointer doubling over
// ds_bpermute (at most six rounds) turns that into the first step that leaves the chunk, and
// the walkers -- one lane per max-level node -- standing in the chunk take it.
__global__ void __launch_bounds__(256) k_chain_exits(const Unit* __restrict__ units, const Seg* __restrict__ segs,
                                                     int32_t nsegs, const int32_t* __restrict__ par,
                                                     const int32_t* __restrict__ exta, const int32_t* __restrict__ qn,
                                                     int32_t* __restrict__ qexit, uint32_t* err) {
  latency_kernel();
  const int l = lane_id();
  const int32_t nw = gridDim.x * 4;
  const int32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wave_id());
  // the wave's segments w, w + nw, ...: 64 descriptions fetched side by side, one per lane
  for (int64_t first = w; first < nsegs; first += (int64_t)64 * nw) {
    const int64_t si = first + (int64_t)l * nw;
    Seg sg = {};
    if (si < nsegs) sg = segs[si];
    const bool live = sg.ord != 0;  // (a unit's first segment has no exit)
    int64_t qa = 0;
    int32_t qprev = 0, q0 = 0;
    if (live) {
      qa = units[sg.unit].a + sg.start;
      qprev = segs[si - 1].qcount;
      q0 = qn[qa];
    }
    for (uint64_t m = __ballot(live); m != 0; m &= m - 1) {
      const int src = __builtin_ctzll(m);
      const int32_t s0 = __builtin_amdgcn_readlane(sg.start, src);
      const int32_t len = __builtin_amdgcn_readlane(sg.len, src);
      const int32_t nq = __builtin_amdgcn_readlane(sg.qcount, src);
      const int32_t qp = __builtin_amdgcn_readlane(qprev, src);
      const int32_t q0u = __builtin_amdgcn_readlane(q0, src);
      const int64_t at = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(qa >> 32), src) << 32) |
                                   (uint32_t)__builtin_amdgcn_readlane((int32_t)qa, src));
      const int32_t* __restrict__ spar = par + (at - s0);  // indexed by row
      const int32_t* __restrict__ sext = exta + (at - s0);
      const int32_t s1 = s0 + len;
      for (int32_t wb = 0; wb < nq; wb += 64) {  // (more than 64 max-level nodes: 64 walkers at a time)
        const bool mine = wb + l < nq;
        int32_t pos = -2;  // a walker's row; negative: -2 - (its exit), the walk is over
        if (mine) {
          pos = nq == 1 ? q0u : qn[at + wb + l];
          if (pos < s0 || pos >= s1) {  // (cannot happen for the kernels' own output)
            raise_error(err, kErrCorrupt);
            pos = -2;
          }
        }
        for (int32_t k = (len - 1) >> 6; k >= 0 && __ballot(pos >= 0) != 0; k -= 4) {
          int32_t pv[4], ev[4];
#pragma unroll
          for (int g = 0; g < 4; g++) {
            const int32_t r = s0 + 64 * (k - g) + l;
            pv[g] = (k - g >= 0 && r < s1) ? spar[r] : -2;
          }
#pragma unroll
          for (int g = 0; g < 4; g++) {  // anchors, where the outside parent's ordinal is past the list
            const int32_t r = s0 + 64 * (k - g) + l;
            ev[g] = (pv[g] < 0 && -2 - pv[g] >= qp) ? sext[r] : 0;
          }
#pragma unroll
          for (int g = 0; g < 4; g++) {
            if (k - g < 0) break;
            const int32_t c0 = s0 + 64 * (k - g);
            int32_t cur = pv[g];
            if (cur < 0 && -2 - cur >= qp) cur = ev[g];
            if (cur == -1 || (cur >= 0 && (cur < s0 || cur >= c0 + l))) {  // (cannot happen: steps lead down)
              raise_error(err, kErrCorrupt);
              cur = -2;
            }
            while (true) {
              const bool inb = cur >= c0;
              if (__ballot(inb) == 0) break;
              const int32_t t = __builtin_amdgcn_ds_bpermute((cur - c0) << 2, cur);
              cur = inb ? t : cur;
            }
            const int32_t t = __builtin_amdgcn_ds_bpermute((pos - c0) << 2, cur);
            pos = pos >= c0 ? t : pos;
            if (__ballot(pos >= 0) == 0) break;
          }
        }
        if (pos >= 0) {  // (a walk that has not ended at the segment's first row: cannot happen)
          raise_error(err, kErrCorrupt);
          pos = -2;
        }
        if (mine) qexit[at + wb + l] = -2 - pos;
      }
    }
  }
}

// Per unit: chain entry index of every segment, last to first; chain length.
__global__ void __launch_bounds__(64) k_chain_entries(Unit* __restrict__ units, int32_t n_units, Seg* __restrict__ segs,
                                                      const int32_t* __restrict__ qexit) {
  latency_kernel();
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
  K = min(K, u.M);  // (always true for a valid permutation; keeps the output layout inside its bound)
  u.K = K;
  u.P = u.M - K;
}

// Mark the chain inside every segment (every row of the segment gets its flag, so the
// flags need no clearing): from its entry node down to relative level 1.  One wave per
// segment walks 64-row chunks of par from the top down (a parent's row is always below its
// child's): the chunk is one coalesced load held one row per lane, each hop inside it is a
// v_readlane instead of a dependent global load, and the chunk's flags are collected in a
// lane mask and stored at once.
__global__ void __launch_bounds__(256) k_chain_mark(const Unit* __restrict__ units, const Seg* __restrict__ segs,
                                                    int32_t nsegs, const int32_t* __restrict__ par,
                                                    const int32_t* __restrict__ qn, uint8_t* __restrict__ chain) {
  latency_kernel();
  const int32_t nw = gridDim.x * 4;
  const int l = lane_id();
  for (int32_t si = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wave_id()); si < nsegs; si += nw) {
    const Seg sg = segs[si];
    const int64_t a = units[sg.unit].a;
    const int32_t s0 = sg.start, s1 = sg.start + sg.len;
    // (kept in a scalar register: the walk below is wave-uniform, one v_readlane per chain node)
    int32_t want = __builtin_amdgcn_readfirstlane(qn[a + s0 + sg.entry]);
    for (int32_t c0 = s0 + ((s1 - 1 - s0) & ~63); c0 >= s0; c0 -= 64) {
      const int32_t r = c0 + l;
      const int32_t pv = (r < s1) ? par[a + r] : 0;
      uint64_t mask = 0;
      while (want >= c0) {
        mask |= 1ull << (want - c0);
        want = __builtin_amdgcn_readlane(pv, want - c0);
      }
      if (r < s1) chain[a + r] = (uint8_t)((mask >> l) & 1);
    }
  }
}

}  // namespace cdcx
