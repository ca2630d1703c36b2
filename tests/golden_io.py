"""Loaders for the committed golden fixtures (tests/golden/*.npz).

The fixtures are data produced by tests/golden/make_golden.py from the
reference itself; nothing here reads /root/reference.
"""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
G1_NAMES = ["g1_c1", "g1_c2", "g1_f9", "g1_dahp", "g1_randwh", "g1_dense", "g1_fixedpath"]


def load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def unpack_obs(packed, shape):
    n = int(np.prod(shape))
    return np.unpackbits(packed)[:n].reshape(shape).astype(np.float32)


class Fuzz:
    """g2_fuzz.npz / g2_evict.npz: ragged one-step scenarios stored flat."""

    def __init__(self, name="g2_fuzz"):
        z = load(name)
        self.count = int(z["count"])
        self.data = {}
        for k in z.files:
            if k.endswith("__len") or k.endswith("__shape") or k == "count":
                continue
            lens = z[k + "__len"]
            shapes = json.loads(str(z[k + "__shape"]))
            flat = z[k]
            offs = np.concatenate([[0], np.cumsum(lens)])
            self.data[k] = [flat[offs[i]:offs[i + 1]].reshape(shapes[i]) for i in range(self.count)]

    def case(self, i):
        return {k: v[i] for k, v in self.data.items()}
