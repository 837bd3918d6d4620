"""Load the committed golden vectors (tests/golden/*.npz) produced by make_golden.py."""
from __future__ import annotations

import glob
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def case_names(prefix: str = ""):
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


class Golden:
    def __init__(self, name: str):
        self.name = name
        with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
            self.z = {k: z[k] for k in z.files}
        self.meta = json.loads(str(self.z["meta"]))

    def has(self, rank, it, key):
        return f"r{rank}_it{it}_{key}" in self.z

    def np(self, rank, it, key):
        return self.z[f"r{rank}_it{it}_{key}"]

    def t(self, rank, it, key):
        a = torch.from_numpy(np.array(self.z[f"r{rank}_it{it}_{key}"]))
        if self.meta.get("dtype") == "bf16" and a.dtype == torch.int16:  # stored bit patterns
            a = a.view(torch.bfloat16)
        return a

    def count(self, rank, it, prefix):
        n = 0
        while f"r{rank}_it{it}_{prefix}{n}" in self.z or f"r{rank}_it{it}_{prefix}{n}_idx" in self.z:
            n += 1
        return n
