// gen.hip -- synthetic rank traces (definition in gen.h) generated in device memory, plus
// the bit-identical host generator used by tests and the CPU baseline.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <numeric>
#include <vector>

#include "cdcx_device.h"
#include "cdcx_kernels.h"
#include "gen.h"

namespace cdcx {

constexpr int kGenTile = 1024;
constexpr int kGenMaxSets = 16;

// Per frame tile: record count and matched count per set.
__global__ void __launch_bounds__(256) k_gen_tile_sums(GenArgs g, int64_t frames_per_rank, int32_t tiles_per_rank,
                                                       int32_t* __restrict__ tsum_rec, int32_t* __restrict__ tsum_set) {
  __shared__ int32_t lds[4];
  const int rr = blockIdx.x / tiles_per_rank, tile = blockIdx.x % tiles_per_rank;
  const int32_t r = g.first_rank + rr;
  const uint64_t seed = gen::rank_seed(r, g.salt);
  const int64_t f0 = (int64_t)tile * kGenTile;
  int32_t rec = 0;
  int32_t per_set[kGenMaxSets] = {0};
  for (int j = threadIdx.x; j < kGenTile; j += 256) {
    const int64_t f = f0 + j;
    if (f >= frames_per_rank) break;
    const gen::Frame fr = gen::frame(seed, g.sh, f);
    rec += fr.unmatched + fr.g;
    per_set[fr.set] += fr.g;
  }
  rec = block_sum<256>(rec, lds);
  if (threadIdx.x == 0) tsum_rec[blockIdx.x] = rec;
  for (int t = 0; t < g.sh.T; t++) {
    int32_t v = block_sum<256>(per_set[t], lds);
    if (threadIdx.x == 0) tsum_set[(int64_t)blockIdx.x * kGenMaxSets + t] = v;
  }
}

// Per rank: exclusive scans of the tile sums (in place).
__global__ void __launch_bounds__(256) k_gen_rank_scan(GenArgs g, int32_t tiles_per_rank, int32_t* __restrict__ tsum_rec,
                                                       int32_t* __restrict__ tsum_set) {
  __shared__ int32_t lds[4];
  const int rr = blockIdx.x;
  int32_t* tr = tsum_rec + (int64_t)rr * tiles_per_rank;
  int32_t* ts = tsum_set + (int64_t)rr * tiles_per_rank * kGenMaxSets;
  for (int t = -1; t < g.sh.T; t++) {
    int32_t run = 0;
    for (int c = 0; c < tiles_per_rank; c += 256) {
      const int i = c + threadIdx.x;
      int32_t v = 0;
      if (i < tiles_per_rank) v = (t < 0) ? tr[i] : ts[(int64_t)i * kGenMaxSets + t];
      int32_t tot;
      const int32_t ex = block_exclusive_scan<256>(v, 0, OpAdd(), lds, &tot) + run;
      if (i < tiles_per_rank) {
        if (t < 0) tr[i] = ex; else ts[(int64_t)i * kGenMaxSets + t] = ex;
      }
      run += tot;
    }
  }
}

// Per frame: record offset and the frame's first matched ordinal within its set.  Frames
// that fit in events_per_rank records raise the rank's frame count / per-set totals.
__global__ void __launch_bounds__(256) k_gen_frames(GenArgs g, int64_t frames_per_rank, int32_t tiles_per_rank,
                                                    const int32_t* __restrict__ tsum_rec, const int32_t* __restrict__ tsum_set,
                                                    int32_t* __restrict__ roff, int32_t* __restrict__ koff,
                                                    int32_t* __restrict__ nframes, int32_t* __restrict__ nmatched,
                                                    int32_t* __restrict__ nrec) {
  __shared__ int32_t lds[4];
  const int rr = blockIdx.x / tiles_per_rank, tile = blockIdx.x % tiles_per_rank;
  const int32_t r = g.first_rank + rr;
  const uint64_t seed = gen::rank_seed(r, g.salt);
  constexpr int PER = kGenTile / 256;
  const int64_t f0 = (int64_t)tile * kGenTile + threadIdx.x * PER;
  gen::Frame fr[PER];
  int32_t rec = 0;
  for (int j = 0; j < PER; j++) {
    const int64_t f = f0 + j;
    fr[j] = (f < frames_per_rank) ? gen::frame(seed, g.sh, f) : gen::Frame{0, 0, 0, 0};
    rec += fr[j].unmatched + fr[j].g;
  }
  int32_t tot;
  int32_t rx = block_exclusive_scan<256>(rec, 0, OpAdd(), lds, &tot) + tsum_rec[blockIdx.x];
  int32_t kx[PER];
  for (int j = 0; j < PER; j++) kx[j] = 0;
  for (int t = 0; t < g.sh.T; t++) {
    int32_t mine = 0;
    for (int j = 0; j < PER; j++) mine += (fr[j].set == t) ? fr[j].g : 0;
    int32_t ex = block_exclusive_scan<256>(mine, 0, OpAdd(), lds, &tot) + tsum_set[(int64_t)blockIdx.x * kGenMaxSets + t];
    for (int j = 0; j < PER; j++) {
      if (fr[j].set == t) kx[j] = ex;
      ex += (fr[j].set == t) ? fr[j].g : 0;
    }
  }
  const int64_t fb = (int64_t)rr * frames_per_rank;
  for (int j = 0; j < PER; j++) {
    const int64_t f = f0 + j;
    if (f >= frames_per_rank) break;
    const int32_t n = fr[j].unmatched + fr[j].g;
    roff[fb + f] = rx;
    koff[fb + f] = kx[j];
    if ((int64_t)rx + n <= g.events) {
      atomicMax(&nframes[rr], (int32_t)(f + 1));
      atomicMax(&nmatched[rr * kGenMaxSets + fr[j].set], kx[j] + fr[j].g);
      atomicMax(&nrec[rr], rx + n);
    }
    rx += n;
  }
}

// Arrival keys of every message of every set (set t's messages at moff[t]).
__global__ void __launch_bounds__(256) k_gen_akeys(GenArgs g, int64_t msgs_per_rank, const int32_t* __restrict__ nmatched,
                                                   int64_t* __restrict__ akey) {
  const int rr = blockIdx.y;
  const int32_t r = g.first_rank + rr;
  const uint64_t seed = gen::rank_seed(r, g.salt);
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int64_t base = 0;
  for (int t = 0; t < g.sh.T; t++) {
    const int32_t n = nmatched[rr * kGenMaxSets + t];
    if (i >= base && i < base + n) {
      akey[(int64_t)rr * msgs_per_rank + i] = gen::message(seed, g.sh, r, t, i - base).akey;
      return;
    }
    base += n;
  }
}

// Arrival position of every message = its rank by (arrival key, m) within its set, found
// by counting inside the +-window_blocks blocks (all earlier blocks arrive before it).
__global__ void __launch_bounds__(256) k_gen_arrival(GenArgs g, int64_t msgs_per_rank, const int32_t* __restrict__ nmatched,
                                                     const int64_t* __restrict__ akey, int32_t* __restrict__ inv) {
  const int rr = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int64_t base = 0;
  for (int t = 0; t < g.sh.T; t++) {
    const int32_t n = nmatched[rr * kGenMaxSets + t];
    if (i >= base && i < base + n) {
      const int64_t m = i - base;
      const int32_t nt = g.sh.senders_of(t);
      const int64_t b = m / nt;
      const int64_t W = gen::window_blocks(g.sh);
      const int64_t* ak = akey + (int64_t)rr * msgs_per_rank + base;
      const int64_t my = ak[m];
      const int64_t blo = b - W > 0 ? b - W : 0;
      int64_t pos = blo * nt;
      const int64_t mhi = (b + W + 1) * nt < n ? (b + W + 1) * nt : n;
      for (int64_t q = blo * nt; q < mhi; q++) {
        const int64_t o = ak[q];
        pos += (o < my) || (o == my && q < m);
      }
      inv[(int64_t)rr * msgs_per_rank + base + pos] = (int32_t)m;
      return;
    }
    base += n;
  }
}

__global__ void __launch_bounds__(256) k_gen_records(GenArgs g, int64_t frames_per_rank, int64_t msgs_per_rank,
                                                     const int32_t* __restrict__ roff, const int32_t* __restrict__ koff,
                                                     const int32_t* __restrict__ nframes, const int32_t* __restrict__ nmatched,
                                                     const int32_t* __restrict__ inv, const int64_t* __restrict__ rec_off,
                                                     int4* __restrict__ rec) {
  const int rr = blockIdx.y;
  const int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (f >= nframes[rr]) return;
  const int32_t r = g.first_rank + rr;
  const uint64_t seed = gen::rank_seed(r, g.salt);
  const gen::Frame fr = gen::frame(seed, g.sh, f);
  const int64_t fb = (int64_t)rr * frames_per_rank;
  int64_t at = rec_off[rr] + roff[fb + f];
  if (fr.unmatched) {
    rec[2 * at] = make_int4(fr.count, 2, 0, 0);
    rec[2 * at + 1] = make_int4(0, 0, 0, fr.set);
    at++;
  }
  int64_t mb = 0;
  for (int t = 0; t < fr.set; t++) mb += nmatched[rr * kGenMaxSets + t];
  const int32_t* iv = inv + (int64_t)rr * msgs_per_rank + mb;
  for (int i = 0; i < fr.g; i++, at++) {
    const int64_t m = iv[koff[fb + f] + i];
    const gen::Msg msg = gen::message(seed, g.sh, r, fr.set, m);
    rec[2 * at] = make_int4(1, 2, 1, msg.src);
    rec[2 * at + 1] = make_int4(i + 1 < fr.g ? 1 : 0, gen::index_of(seed, f, i), msg.clock, fr.set);
  }
}

// Host twin (tests, CPU baseline): the same stream, sequentially.
std::vector<int32_t> generate_host(const GenArgs& g, int32_t r) {
  const uint64_t seed = gen::rank_seed(r, g.salt);
  std::vector<gen::Frame> frames;
  std::vector<int32_t> n(g.sh.T, 0);
  int64_t total = 0;
  for (int64_t f = 0;; f++) {
    const gen::Frame fr = gen::frame(seed, g.sh, f);
    if (total + fr.unmatched + fr.g > g.events) break;
    total += fr.unmatched + fr.g;
    n[fr.set] += fr.g;
    frames.push_back(fr);
  }
  std::vector<std::vector<int32_t>> order(g.sh.T);
  for (int t = 0; t < g.sh.T; t++) {
    std::vector<int64_t> ak(n[t]);
    for (int64_t m = 0; m < n[t]; m++) ak[m] = gen::message(seed, g.sh, r, t, m).akey;
    order[t].resize(n[t]);
    std::iota(order[t].begin(), order[t].end(), 0);
    std::stable_sort(order[t].begin(), order[t].end(), [&](int32_t x, int32_t y) { return ak[x] < ak[y]; });
  }
  std::vector<int32_t> out;
  out.reserve(8 * total);
  std::vector<int32_t> k(g.sh.T, 0);
  for (int64_t f = 0; f < (int64_t)frames.size(); f++) {
    const gen::Frame& fr = frames[f];
    if (fr.unmatched) {
      const int32_t rr[8] = {fr.count, 2, 0, 0, 0, 0, 0, fr.set};
      out.insert(out.end(), rr, rr + 8);
    }
    for (int i = 0; i < fr.g; i++) {
      const gen::Msg msg = gen::message(seed, g.sh, r, fr.set, order[fr.set][k[fr.set]++]);
      const int32_t rr[8] = {1, 2, 1, msg.src, i + 1 < fr.g ? 1 : 0, gen::index_of(seed, f, i), msg.clock, fr.set};
      out.insert(out.end(), rr, rr + 8);
    }
  }
  return out;
}

}  // namespace cdcx
