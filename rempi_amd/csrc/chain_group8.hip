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
constexpr int kRing8 = 64;  // rows of {par, column} per group in LDS
constexpr int kLongSeg = 1536;  // events: segments from here on run at raised wave priority

__device__ __forceinline__ int lane8() { return threadIdx.x & 7; }
__device__ __forceinline__ int base8() { return threadIdx.x & 56; }
__device__ __forceinline__ uint32_t ballot8(bool p) {
  return (uint32_t)((unsigned long long)__builtin_amdgcn_ballot_w64(p) >> base8()) & 0xFFu;
}
// value of the group's lane 0
__device__ __forceinline__ int32_t first8(int32_t v) {
  int32_t t = __builtin_amdgcn_update_dpp(0, v, 0x150, 0xf, 0x3, false);  // row_newbcast:0 -> lanes 0-7 of the row
  return __builtin_amdgcn_update_dpp(t, v, 0x158, 0xf, 0xC, false);       // row_newbcast:8 -> lanes 8-15
}
// value of group lane l (l group-uniform)
__device__ __forceinline__ int32_t at8(int32_t v, int32_t l) { return __builtin_amdgcn_ds_bpermute((base8() + l) << 2, v); }
// lane j <- lane j+1 (the group's lane 7 receives the neighbouring group's lane 0, or keeps its value)
__device__ __forceinline__ int32_t next8(int32_t v) { return __builtin_amdgcn_update_dpp(v, v, 0x101, 0xf, 0xf, false); }
// lane j <- lane j-1 (the group's lane 0 receives the neighbouring group's lane 7, or keeps its value)
__device__ __forceinline__ int32_t prev8(int32_t v) { return __builtin_amdgcn_update_dpp(v, v, 0x111, 0xf, 0xf, false); }
__device__ __forceinline__ int32_t push8(int32_t v, int32_t dst) { return __builtin_amdgcn_ds_permute((base8() + dst) << 2, v); }
__device__ __forceinline__ uint32_t below(int j) { return (1u << j) - 1u; }
}  // namespace

__global__ void __launch_bounds__(256) k_chain_grp8(const Unit* __restrict__ units, Seg* __restrict__ segs,
                                                    const int32_t* __restrict__ list, const int32_t* __restrict__ nlist_p,
                                                    const int32_t* __restrict__ cord, const int32_t* __restrict__ opn,
                                                    int32_t* __restrict__ par, int32_t* __restrict__ exta,
                                                    int32_t* __restrict__ topg, int32_t* __restrict__ qn,
                                                    int32_t* __restrict__ ovf, int32_t* __restrict__ novf, uint32_t* err) {
  constexpr int G = G8;
  constexpr int kGroups = 256 / G;
  constexpr int R = kRing8;
  __shared__ int32_t next_j;
  __shared__ int2 ring_all[kGroups][R];   // {par, column} of row r at [r % R]
  __shared__ int32_t comp_all[kGroups][3 * 16];  // sweep compaction of a list that uses the B slots
  int2* ring = ring_all[threadIdx.x / G];
  int32_t* comp = comp_all[threadIdx.x / G];
  if (threadIdx.x == 0) next_j = 0;
  __syncthreads();

  const int j = lane8();
  const int32_t nlist = *nlist_p;
  // group-uniform state
  int32_t si = -1, s0 = 0, s1 = 0, ord = 0;
  int64_t a = 0;
  int32_t i = 0, nl = 0, lmax = 0, nrel1 = 0, qcnt = 0, cb = 0;
  bool islong = false;
  // lane state: leaf slots j (A) and 8 + j (B), top of level lmax - j, row windows, parent buffer
  int32_t lid = 0, llv = 0, lcol = 0, lidB = 0, llvB = 0, lcolB = 0;
  int32_t top = 0, cw0 = 0, cw1 = 0, ow0 = 0, ow1 = 0, pval = 0;

  auto node = [&](int32_t x) -> int2 {  // {par, column} of row x < i of this segment
    if (x >= i - R) return ring[x & (R - 1)];
    return make_int2(par[a + x], cord[a + x]);
  };

  while (true) {
    if (i >= s1) {
      if (si >= 0) {
        if (cb + j < s1) par[a + cb + j] = pval;
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
      si = list[kk];
      const Seg sg = segs[si];
      a = units[sg.unit].a;
      s0 = sg.start;
      s1 = sg.start + sg.len;
      ord = sg.ord;
      i = cb = s0;
      nl = lmax = nrel1 = qcnt = 0;
      // The kernel ends when its longest segments end, and they share their SIMD with other
      // waves all the way: a wave that runs one of them issues ahead of the others.
      islong = sg.len >= kLongSeg;
      if (__builtin_amdgcn_ballot_w64(islong) != 0)
        __builtin_amdgcn_s_setprio(3);
      else
        __builtin_amdgcn_s_setprio(0);
      cw0 = (s0 + j < s1) ? cord[a + s0 + j] : 0;
      cw1 = (s0 + G + j < s1) ? cord[a + s0 + G + j] : 0;
      ow0 = (s0 + j < s1) ? opn[a + s0 + j] : 0;
      ow1 = (s0 + G + j < s1) ? opn[a + s0 + G + j] : 0;
    } else if (i - cb == G) {  // flush this window's parents, slide the row windows
      par[a + cb + j] = pval;
      cb += G;
      cw0 = cw1;
      cw1 = (cb + G + j < s1) ? cord[a + cb + G + j] : 0;
      ow0 = ow1;
      ow1 = (cb + G + j < s1) ? opn[a + cb + G + j] : 0;
    }
    const int32_t t = i - cb;
    const int32_t c = first8(cw0);     // column of row i
    cw0 = next8(cw0);
    const int32_t open = first8(ow0);  // first column not taken by rows < i
    ow0 = next8(ow0);
    // does any group of this wave use its B slots in this iteration?
    const bool useB = __builtin_amdgcn_ballot_w64(nl > G) != 0;

    // ---- k*: highest level whose top column is smaller than c ---------------------------
    const uint32_t tm = ballot8(j < lmax && top < c);
    int32_t ks = 0;
    if (tm) {
      ks = lmax - (__ffs(tm) - 1);
    } else if (lmax > G) {  // below the register tops: binary search the spilled levels
      int32_t lo = 1, hi = lmax - G;
      while (lo <= hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (topg[a + s0 + mid - 1] < c) {
          ks = mid;
          lo = mid + 1;
        } else {
          hi = mid - 1;
        }
      }
    }

    // ---- parent --------------------------------------------------------------------------
    int32_t pv, pslot = -1;
    if (ks >= 1) {
      uint32_t eq = ballot8(j < nl && llv == ks && lcol < c);
      uint32_t gt = ballot8(j < nl && llv > ks);
      if (useB) {
        eq |= ballot8(j + G < nl && llvB == ks && lcolB < c) << G;
        gt |= ballot8(j + G < nl && llvB > ks) << G;
      }
      const int wa = eq ? __ffs(eq) - 1 : 2 * G;
      const uint32_t need = gt & below(wa);
      int win = wa;
      int32_t anc = -1;
      bool interior = false;
      if (need) {
        // every slot before wa holding a deeper leaf climbs to its level-k* ancestor at once
        const bool mine = (need >> j) & 1u;
        int32_t x = lid, col = 0x7fffffff;
        if (mine) {
          for (int32_t d = llv - ks; d > 0; d--) x = node(x).x;
          col = node(x).y;
        }
        uint32_t ok = ballot8(mine && col < c);
        int32_t xB = lidB;
        if (useB) {
          const bool mineB = (need >> (j + G)) & 1u;
          int32_t colB = 0x7fffffff;
          if (mineB) {
            for (int32_t d = llvB - ks; d > 0; d--) xB = node(xB).x;
            colB = node(xB).y;
          }
          ok |= ballot8(mineB && colB < c) << G;
        }
        if (ok) {
          win = __ffs(ok) - 1;
          interior = true;
          const int32_t aA = at8(x, win & 7), aB = at8(xB, win & 7);
          anc = win < G ? aA : aB;
        }
      }
      if (win >= 2 * G) {
        raise_error(err, kErrCorrupt);  // cannot happen for a valid permutation
        win = 0;
      }
      if (interior) {
        pv = anc;
      } else {
        const int32_t pA = at8(lid, win & 7);
        pv = pA;
        if (useB) {
          const int32_t pB = at8(lidB, win & 7);
          pv = win < G ? pA : pB;
        }
        pslot = win;
      }
    } else if (ord == 0) {
      pv = -1;  // first segment: level 1 hangs off the root
    } else {
      // outside parent, resolved at stitching from (ordinal, first leaf) -- chain.hip
      pv = -2 - nrel1;
      const int32_t f = first8(lid);
      if (j == 0) exta[a + i] = nl > 0 ? f : -1;
      nrel1++;
    }
    if (j == t) pval = pv;
    if (j == 0) ring[i & (R - 1)] = make_int2(pv, c);

    // ---- tops ------------------------------------------------------------------------------
    const int32_t k = ks + 1;
    const bool grow = k > lmax;
    if (grow && j == G - 1 && lmax - (G - 1) >= 1) topg[a + s0 + (lmax - (G - 1)) - 1] = top;
    if (!grow && lmax - k >= G && j == 0) topg[a + s0 + k - 1] = c;
    const int32_t tshift = prev8(top);
    top = grow ? ((j == 0) ? c : tshift) : ((j == lmax - k) ? c : top);
    qcnt = grow ? 0 : qcnt;
    lmax = grow ? k : lmax;
    if (k == lmax && j == 0) qn[a + s0 + qcnt] = i;
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
        const bool dropB = pslot >= 0 && j + G >= pslot;
        lidB = dropB ? nidB : lidB;
        llvB = dropB ? nlvB : llvB;
        lcolB = dropB ? ncolB : lcolB;
      }
      const bool drop = pslot >= 0 && j >= pslot;
      lid = drop ? nid : lid;
      llv = drop ? nlv : llv;
      lcol = drop ? ncol : lcol;
      nl -= (pslot >= 0) ? 1 : 0;
    }
    // (the sweep comes before the append: the new node, on column `open` itself, is never swept)
    if (c == open) {
      uint32_t dead = ballot8(j < nl && lcol < open);
      if (!useB) {
        if (dead) {
          const int32_t dst = (j < nl && !((dead >> j) & 1u)) ? j - __popc(dead & below(j)) : G - 1;
          lid = push8(lid, dst);
          llv = push8(llv, dst);
          lcol = push8(lcol, dst);
          nl -= __popc(dead);
        }
      } else {
        dead |= ballot8(j + G < nl && lcolB < open) << G;
        if (dead) {
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
    if (nl == 2 * G) {  // leaf list outgrows the group: hand the segment to the next tier
      if (j == 0) ovf[atomicAdd(novf, 1)] = si;
      si = -1;
      i = s1 - 1;  // the rest of this iteration runs on junk state and ends the segment
      nl = 0;
    }
    if (j == nl) {
      lid = i;
      llv = k;
      lcol = c;
    }
    if (j + G == nl) {
      lidB = i;
      llvB = k;
      lcolB = c;
    }
    nl++;

    i++;
  }
}

}  // namespace cdcx
