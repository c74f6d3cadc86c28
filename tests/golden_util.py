"""Loading the committed golden fixtures (data only, numpy allow_pickle=False)."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def names():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return sorted(json.load(f))


def load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["max_len"] = int(d["max_len"])
    d["ref_failed"] = bool(int(d["ref_failed"]))
    if not d["ref_failed"]:
        d["rempi"] = d["rempi"].tobytes()
        d["tables"] = d["tables"].tobytes()
    return d


def all_files():
    return glob.glob(os.path.join(GOLDEN, "*.npz"))


def basic_names():
    """Fixtures of the basic -> CDC transcoder (tests/golden/make_basic_golden.py)."""
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "basic_*.npz")))


def load_basic(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["max_len"] = int(d["max_len"])
    d["basic"] = d["basic"].tobytes()
    d["basic_gz"] = d["basic_gz"].tobytes()
    d["rempi"] = d["rempi"].tobytes()
    return d


def gzip_names():
    """Fixtures of the REMPI_GZIP=1 stage (tests/golden/make_gzip_golden.py)."""
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "gzip_*.npz")))


def load_gzip(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["max_len"] = int(d["max_len"])
    for k in ("rempi", "rempi_gz", "tables"):
        d[k] = d[k].tobytes()
    return d


def rep_names():
    """Fixtures of the rep encoder, REMPI_ENCODE=7 (tests/golden/make_rep_golden.py)."""
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "rep_*.npz")))


def load_rep(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["max_len"] = int(d["max_len"])
    for k in ("rempi_rep", "tables"):
        d[k] = d[k].tobytes()
    return d


def footer_names():
    """Fixtures of the footer's matching-set-id map (tests/golden/make_footer_golden.py)."""
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "footer_*.npz")))


def load_footer(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["max_len"] = int(d["max_len"])
    d["rempi"] = d["rempi"].tobytes()
    return d
