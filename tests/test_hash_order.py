"""The libstdc++ unordered_{map,set} iteration-order emulation used on the device
(rempi_amd/csrc/hash_order.h) against the live containers of this image's libstdc++
(called through the oracle library)."""
import os
import subprocess
import tempfile

import numpy as np
import pytest

import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DRIVER = r"""
#include "hash_order.h"
#include <cstdio>
#include <vector>
int main() {
  long n; std::vector<unsigned long long> out;
  while (scanf("%ld", &n) == 1) {
    std::vector<long long> k(n);
    for (auto& x : k) scanf("%lld", &x);
    std::vector<uint64_t> key(n + 1); std::vector<int32_t> nx(n + 1), bk(cdcx::hash_bucket_capacity(n) + 1);
    cdcx::HashOrder h; h.init(key.data(), nx.data(), bk.data());
    for (auto x : k) if (!h.contains((uint64_t)x)) h.insert_new((uint64_t)x);
    printf("%d", h.size);
    for (int p = h.head; p != -1; p = h.next[p]) printf(" %lld", (long long)h.key[p]);
    printf("\n");
  }
}
"""


@pytest.fixture(scope="module")
def driver():
    d = tempfile.mkdtemp()
    src = os.path.join(d, "ho.cpp")
    with open(src, "w") as f:
        f.write(DRIVER)
    exe = os.path.join(d, "ho")
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "rempi_amd", "csrc"), src, "-o", exe])
    return exe


def _run(exe, seqs):
    inp = "".join(f"{len(s)} " + " ".join(str(int(x)) for x in s) + "\n" for s in seqs)
    out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout.strip().split("\n")
    return [list(map(int, line.split()))[1:] for line in out]


def test_map_order_matches_libstdcxx(driver):
    rng = np.random.default_rng(3)
    seqs = []
    for t in range(300):
        n = int(rng.integers(0, 400 if t < 280 else 6000))
        hi = [64, 1100, 1 << 40][t % 3]
        seqs.append(rng.integers(0, hi, size=n))
    got = _run(driver, seqs)
    for s, g in zip(seqs, got):
        assert g == list(O.umap_order(s))


def test_set_int_order_matches_libstdcxx(driver):
    """unordered_set<int> (footer): same hash (identity, sign-extended), same table."""
    rng = np.random.default_rng(4)
    seqs = [rng.integers(0, 5000, size=int(rng.integers(0, 3000))) for _ in range(40)]
    got = _run(driver, seqs)
    for s, g in zip(seqs, got):
        assert g == list(O.uset_int_order(s.astype(np.int32)))
