// chain_group.hip -- the segment chain simulation (chain.hip) with one segment per group of
// G lanes instead of one per lane.
//
// Same rule and the same outputs as k_chain_seg (par, exta, topg, qn, segs[].lmax/qcount),
// but the per-segment state lives *across* the G lanes of a group:
//   lane j holds leaf slot j (leaves in creation order: id, level, column),
//   lane j holds the patience top of level lmax - j (the top G levels; lower ones spill),
//   lane j holds cord and opn (first untaken column, k_cuts) of row base + j (two G-row
//   windows each, prefetched),
//   lane j buffers par of row cb + j until the window is flushed (coalesced store).
// Every leaf-list operation of the lane kernel (first qualifying slot, erase, append, sweep)
// becomes one or two lane-parallel instructions plus a ballot, so an event costs ~70 VALU
// instructions of latency instead of ~1000; the long segments that set the kernel's tail
// finish ~10x sooner.  G = 16 maps a group onto one DPP row (row_shl / row_shr /
// row_newbcast); G = 64 is a whole wave (wave_shl / wave_shr / readlane) for segments whose
// leaf list outgrows 16 slots.  A group whose leaf list outgrows G slots abandons the
// segment and queues it for the next tier (G = 64, then the lane kernel's exact
// global-memory path); the tiers rewrite every output of the segment from scratch.
//
// Parent climbs read par/column of recent rows from a per-group LDS ring (rows
// [i - kRing, i)), older rows from global memory (flushed windows).
#include <hip/hip_runtime.h>

#include "cdcx_device.h"
#include "cdcx_kernels.h"

namespace cdcx {

namespace {

template <int G>
struct Grp;

template <>
struct Grp<16> {
  using Mask = uint32_t;
  __device__ static __forceinline__ int lane() { return threadIdx.x & 15; }
  __device__ static __forceinline__ int base() { return threadIdx.x & 48; }
  __device__ static __forceinline__ Mask ballot(bool p) {
    return (Mask)((unsigned long long)__builtin_amdgcn_ballot_w64(p) >> base()) & 0xFFFFu;
  }
  // value of group lane 0 (DPP row_newbcast:0)
  __device__ static __forceinline__ int32_t first(int32_t v) { return __builtin_amdgcn_update_dpp(0, v, 0x150, 0xf, 0xf, false); }
  // value of group lane l (l group-uniform)
  __device__ static __forceinline__ int32_t at(int32_t v, int32_t l) { return __builtin_amdgcn_ds_bpermute((base() + l) << 2, v); }
  // lane j <- lane j+1 (row_shl:1); the last lane keeps its value
  __device__ static __forceinline__ int32_t from_next(int32_t v) { return __builtin_amdgcn_update_dpp(v, v, 0x101, 0xf, 0xf, false); }
  // lane j <- lane j-1 (row_shr:1); lane 0 keeps its value
  __device__ static __forceinline__ int32_t from_prev(int32_t v) { return __builtin_amdgcn_update_dpp(v, v, 0x111, 0xf, 0xf, false); }
  // lane j's value lands in group lane dst (every lane must target a distinct lane or junk)
  __device__ static __forceinline__ int32_t push(int32_t v, int32_t dst) { return __builtin_amdgcn_ds_permute((base() + dst) << 2, v); }
  __device__ static __forceinline__ int ffs(Mask m) { return __ffs(m) - 1; }
  __device__ static __forceinline__ int popc(Mask m) { return __popc(m); }
  __device__ static __forceinline__ Mask below(int j) { return (1u << j) - 1u; }
  __device__ static __forceinline__ bool bit(Mask m, int j) { return (m >> j) & 1u; }
};

template <>
struct Grp<64> {
  using Mask = unsigned long long;
  __device__ static __forceinline__ int lane() { return threadIdx.x & 63; }
  __device__ static __forceinline__ int base() { return 0; }
  __device__ static __forceinline__ Mask ballot(bool p) { return (Mask)__builtin_amdgcn_ballot_w64(p); }
  __device__ static __forceinline__ int32_t first(int32_t v) { return __builtin_amdgcn_readlane(v, 0); }
  __device__ static __forceinline__ int32_t at(int32_t v, int32_t l) {
    return __builtin_amdgcn_readlane(v, __builtin_amdgcn_readfirstlane(l));
  }
  __device__ static __forceinline__ int32_t from_next(int32_t v) { return __builtin_amdgcn_update_dpp(v, v, 0x130, 0xf, 0xf, false); }
  __device__ static __forceinline__ int32_t from_prev(int32_t v) { return __builtin_amdgcn_update_dpp(v, v, 0x138, 0xf, 0xf, false); }
  __device__ static __forceinline__ int32_t push(int32_t v, int32_t dst) { return __builtin_amdgcn_ds_permute(dst << 2, v); }
  __device__ static __forceinline__ int ffs(Mask m) { return __ffsll(m) - 1; }
  __device__ static __forceinline__ int popc(Mask m) { return __popcll(m); }
  __device__ static __forceinline__ Mask below(int j) { return j >= 64 ? ~0ull : (1ull << j) - 1ull; }
  __device__ static __forceinline__ bool bit(Mask m, int j) { return (m >> j) & 1ull; }
};

template <int G>
constexpr int ring_rows() { return G == 16 ? 128 : 256; }

}  // namespace

template <int G>
__global__ void __launch_bounds__(256) k_chain_grp(const Unit* __restrict__ units, Seg* __restrict__ segs,
                                                   const int32_t* __restrict__ list, const int32_t* __restrict__ nlist_p,
                                                   const int32_t* __restrict__ cord, const int32_t* __restrict__ opn,
                                                   int32_t* __restrict__ par, int32_t* __restrict__ exta,
                                                   int32_t* __restrict__ topg, int32_t* __restrict__ qn,
                                                   int32_t* __restrict__ ovf, int32_t* __restrict__ novf, uint32_t* err) {
  using Gr = Grp<G>;
  using Mask = typename Gr::Mask;
  constexpr int kGroups = 256 / G;
  constexpr int R = ring_rows<G>();
  if (G == 64) latency_kernel();  // the second tier: a handful of segments, one per wave
  __shared__ int32_t next_j;
  __shared__ int2 ring_all[kGroups][R];  // {par, column} of row r at [r % R]
  int2* ring = ring_all[threadIdx.x / G];
  if (threadIdx.x == 0) next_j = 0;
  __syncthreads();

  const int j = Gr::lane();
  const int32_t nlist = *nlist_p;
  // group-uniform state
  int32_t si = -1, s0 = 0, s1 = 0, ord = 0;
  int64_t a = 0;
  int32_t i = 0, nl = 0, lmax = 0, nrel1 = 0, qcnt = 0, cb = 0;
  // lane state
  int32_t lid = 0, llv = 0, lcol = 0, top = 0, cw0 = 0, cw1 = 0, ow0 = 0, ow1 = 0, pval = 0;

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
      k = Gr::first(k);
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
      cw0 = (s0 + j < s1) ? cord[a + s0 + j] : 0;
      cw1 = (s0 + G + j < s1) ? cord[a + s0 + G + j] : 0;
      ow0 = (s0 + j < s1) ? opn[a + s0 + j] : 0;
      ow1 = (s0 + G + j < s1) ? opn[a + s0 + G + j] : 0;
      // (no `continue`: the first event follows in this iteration; a single loop back-edge
      // keeps the compiler from copying the whole loop state through extra phi blocks)
    } else if (i - cb == G) {  // flush this window's parents, slide the cord window
      par[a + cb + j] = pval;
      cb += G;
      cw0 = cw1;
      cw1 = (cb + G + j < s1) ? cord[a + cb + G + j] : 0;
      ow0 = ow1;
      ow1 = (cb + G + j < s1) ? opn[a + cb + G + j] : 0;
    }
    const int32_t t = i - cb;
    // c of row i: lane 0 of the window, which shifts down one lane per row (DPP, no LDS trip)
    const int32_t c = Gr::first(cw0);
    cw0 = Gr::from_next(cw0);
    // first column not taken by rows < i, likewise
    const int32_t open = Gr::first(ow0) < 0 ? c : -1;  // c when row i is open (k_cuts)
    ow0 = Gr::from_next(ow0);

    // ---- k*: highest level whose top column is smaller than c ---------------------------
    const Mask tm = Gr::ballot(j < lmax && top < c);
    int32_t ks = 0;
    if (tm) {
      ks = lmax - Gr::ffs(tm);
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
      const bool live = j < nl;
      const Mask eq = Gr::ballot(live && llv == ks && lcol < c);
      const Mask gt = Gr::ballot(live && llv > ks);
      const int wa = eq ? Gr::ffs(eq) : G;
      const Mask need = gt & Gr::below(wa);
      int win = wa;
      int32_t anc = -1;
      bool interior = false;
      if (need) {
        // every slot before wa holding a deeper leaf climbs to its level-k* ancestor at once
        const bool mine = Gr::bit(need, j);
        int32_t x = lid, col = 0x7fffffff;
        if (mine) {
          for (int32_t d = llv - ks; d > 0; d--) x = node(x).x;
          col = node(x).y;
        }
        const Mask ok = Gr::ballot(mine && col < c);
        if (ok) {
          win = Gr::ffs(ok);
          interior = true;
          anc = Gr::at(x, win);
        }
      }
      if (win >= G) {
        raise_error(err, kErrCorrupt);  // cannot happen for a valid permutation
        win = 0;
      }
      if (interior) {
        pv = anc;
      } else {
        pv = Gr::at(lid, win);
        pslot = win;
      }
    } else if (ord == 0) {
      pv = -1;  // first segment: level 1 hangs off the root
    } else {
      // outside parent, resolved at stitching from (ordinal, first leaf) -- chain.hip
      pv = -2 - nrel1;
      const int32_t f = Gr::first(lid);
      if (j == 0) exta[a + i] = nl > 0 ? f : -1;
      nrel1++;
    }
    if (j == t) pval = pv;
    if (j == 0) ring[i & (R - 1)] = make_int2(pv, c);

    // ---- tops ------------------------------------------------------------------------------
    // (the common updates below are predicated selects on group-uniform conditions rather
    // than branches: the four groups of a wave rarely agree, and a divergent branch costs
    // the CU-shared scalar unit more than the few vector ops it would skip)
    const int32_t k = ks + 1;
    const bool grow = k > lmax;
    if (grow && j == G - 1 && lmax - (G - 1) >= 1) topg[a + s0 + (lmax - (G - 1)) - 1] = top;
    if (!grow && lmax - k >= G && j == 0) topg[a + s0 + k - 1] = c;
    const int32_t tshift = Gr::from_prev(top);
    top = grow ? ((j == 0) ? c : tshift) : ((j == lmax - k) ? c : top);
    qcnt = grow ? 0 : qcnt;
    lmax = grow ? k : lmax;
    if (k == lmax && j == 0) qn[a + s0 + qcnt] = i;
    qcnt += (k == lmax) ? 1 : 0;

    // ---- leaves: drop the adopted one, append the new node, sweep ------------------------
    {
      const int32_t nid = Gr::from_next(lid), nlv = Gr::from_next(llv), ncol = Gr::from_next(lcol);
      const bool drop = pslot >= 0 && j >= pslot;
      lid = drop ? nid : lid;
      llv = drop ? nlv : llv;
      lcol = drop ? ncol : lcol;
      nl -= (pslot >= 0) ? 1 : 0;
    }
    // (the sweep comes before the append: the new node, on column `open` itself, is never
    // swept, and a list that is full only until the sweep need not leave the tier)
    if (c == open) {
      const Mask dead = Gr::ballot(j < nl && lcol < open);
      if (dead) {
        const int32_t dst = (j < nl && !Gr::bit(dead, j)) ? j - Gr::popc(dead & Gr::below(j)) : G - 1;
        lid = Gr::push(lid, dst);
        llv = Gr::push(llv, dst);
        lcol = Gr::push(lcol, dst);
        nl -= Gr::popc(dead);
      }
    }
    if (nl == G) {  // leaf list outgrows the group: hand the segment to the next tier
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
    nl++;

    i++;
  }
}

template __global__ void k_chain_grp<16>(const Unit*, Seg*, const int32_t*, const int32_t*, const int32_t*, const int32_t*,
                                         int32_t*, int32_t*, int32_t*, int32_t*, int32_t*, int32_t*, uint32_t*);
template __global__ void k_chain_grp<64>(const Unit*, Seg*, const int32_t*, const int32_t*, const int32_t*, const int32_t*,
                                         int32_t*, int32_t*, int32_t*, int32_t*, int32_t*, int32_t*, uint32_t*);

}  // namespace cdcx
