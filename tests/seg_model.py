"""Host model of the permutation rebuild's pair-segment tier (rempi_amd/csrc/decode.hip:
k_dec_pair_scan, k_dec_perm_seg<true>, k_dec_perm_check), statement by statement but with plain
Python lists.  Test infrastructure: tests/test_seg_model.py runs it against the oracle's
cdc_prepare_decode_indices to pin the argument the tier rests on -- a unit whose segments all
finish and all pass the check has exactly the sequential replay's permutation -- on inputs the
GPU tests also use; the product never imports it.

The list of rempi_encoder_cdc.cpp:1301-1386 is [0..M); pair (id, delay) takes `id` out and puts
it back `delay` places from where it was.  A segment owns the pairs [ka, ke) and the list
positions [own, cap).  It starts from the untouched list, replays the WARM pairs before `ka`
without writing (pairs that do not fit its window are skipped), and the W positions from `own`
are then compared with the same positions of the state its predecessor ended in."""
from __future__ import annotations

W, AHEAD = 128, 56            # window slots, room kept behind an untouched id
PAIRS, WARM, DELTA = 2048, 128, 32
MAXP = 262144
NOCAP = 0x7FFFFFF0


def nseg(P):
    return 1 if (P <= PAIRS or P > MAXP) else (P + PAIRS - 1) // PAIRS


def seg_floor(v):
    return max(0, v - DELTA) & ~15


def layout(ids):
    """k_dec_pair_scan: (ka, ke, own, cap, base0) of every segment from the suffix minima of the
    ids, taken every WARM pairs."""
    P = len(ids)
    n = nseg(P)
    if n == 1:
        return [(0, P, 0, NOCAP, 0)]
    nb = (P + WARM - 1) // WARM
    bmin = [min(int(v) if -2**31 <= int(v) < 2**31 else ((int(v) + 2**31) % 2**32) - 2**31
                for v in ids[b * WARM:(b + 1) * WARM]) for b in range(nb)]
    for b in range(nb - 2, -1, -1):
        bmin[b] = min(bmin[b], bmin[b + 1])
    out = []
    for s in range(n):
        ka = s * PAIRS
        out.append((ka, min(P, ka + PAIRS),
                    seg_floor(bmin[ka // WARM]) if s else 0,
                    min(NOCAP, seg_floor(bmin[(ka + PAIRS) // WARM])) if s + 1 < n else NOCAP,
                    seg_floor(bmin[(ka - WARM) // WARM]) if s else 0))
    return out


class Group:
    """One 16-lane group of k_dec_perm_seg: the window [base, base + W) of the list; every
    position from base + W on holds its own index."""

    def __init__(self, M, base0):
        self.M = M
        self.base = base0
        self.win = list(range(base0, base0 + W))
        self.out = {}  # list position -> element, as written to cinv (perm is its inverse)

    def slide(self, write):
        if write:
            for j in range(16):
                if self.win[j] < self.M:
                    self.out[self.base + j] = self.win[j]
        self.win = self.win[16:] + list(range(self.base + W, self.base + W + 16))
        self.base += 16

    def step(self, x, d, warm, lim):
        """One pair; False if it does not fit (skipped in the replay, fails the unit otherwise)."""
        if x >= self.base + W:
            while x >= self.base + W - AHEAD and self.base + 16 <= lim:
                self.slide(not warm)
        if x not in self.win:  # behind the window, past it, or not a list element
            return False
        p = self.win.index(x)
        t = p + d
        if t < 0 or self.base + t > self.M - 1:
            return False
        while t > W - 1:
            if p < 16 or self.base + 16 > lim:
                return False
            self.slide(not warm)
            p -= 16
            t -= 16
        self.win.pop(p)
        self.win.insert(t, x)
        return True


def run_segment(ids, dl, M, seg, first, from_state=None):
    """-> (ok, written positions, state it started its own pairs from, state it ends in);
    from_state: run again from this state at `own` instead of the replay (k_dec_perm_seg<2>)"""
    ka, ke, own, cap, base0 = seg
    g = Group(M, base0)
    start = None
    if from_state is not None:
        g.base = own
        g.win = list(from_state)
        start = list(from_state)
    elif not first:
        for k in range(ka - WARM, ka):
            g.step(int(ids[k]), int(dl[k]), True, own)
        while g.base < own:
            g.slide(False)
        start = list(g.win)
    for k in range(ka, ke):
        x = int(ids[k])
        if not (0 <= x < M) or not g.step(x, int(dl[k]), False, cap):
            return False, {}, start, None
    lim = min(M, cap)
    for s in range(W):
        if g.win[s] < M and g.base + s < lim:
            g.out[g.base + s] = g.win[s]
    for q in range(g.base + W, lim):
        g.out[q] = q
    end = None
    if cap != NOCAP:
        end = [g.win[cap + q - g.base] if cap + q < g.base + W else cap + q for q in range(W)]
    return True, g.out, start, end


def rebuild(ids, dl, M, stats=None):
    """The tier on one unit: perm (list) if every segment finishes and starts from the state its
    predecessor ended in -- after running again from that state where its replay gave another
    (the device gives up after two rounds of such reruns; here every segment gets one, in order,
    which is where those rounds end up when they suffice) -- else None (the unit goes to the
    whole-unit tiers).  perm is read off cinv, as k_dec_perm_inv does after reruns."""
    segs = layout(ids)
    cinv = {}
    prev_end = None
    for s, seg in enumerate(segs):
        ok, out, start, end = run_segment(ids, dl, M, seg, s == 0)
        if ok and s > 0 and start != prev_end:
            if stats is not None:
                stats["reruns"] = stats.get("reruns", 0) + 1
            ok, out, start, end = run_segment(ids, dl, M, seg, False, from_state=prev_end)
        if not ok:
            return None
        cinv.update(out)
        prev_end = end
    if sorted(cinv) != list(range(M)):
        return None  # (cannot happen for a unit that passed; kept as a check of the model itself)
    perm = [0] * M
    for pos, v in cinv.items():
        perm[v] = pos
    return perm
