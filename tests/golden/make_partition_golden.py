"""Golden vectors of the reference's data partitioner (run in the build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_partition_golden.py

The drivers that hold ``allocate_dataset`` cannot be imported (module-scope MNIST download,
torchvision / fedlab missing: SURVEY 8c), so this script parses the two reference source files with
``ast``, compiles ONLY the ``allocate_dataset`` (+ ``del_tensor_ele``) function definitions and runs
them in a namespace holding the driver globals they read (``rd`` seeded as the drivers seed it,
``num_workers``, ``num_class``, ``num_sample``, ``datasets``) on synthetic label vectors.  The data
tensors carry each sample's original index, so every shard the reference builds is recorded as a
list of original indices.  Output: tests/golden/partition.json (data only).
"""
import ast
import copy
import json
import os
import sys
from random import Random

sys.dont_write_bytecode = True

import numpy as np
import torch

REF = os.environ.get("CGL_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def _functions(relpath, names):
    src = open(os.path.join(REF, relpath)).read()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names]
    assert len(keep) == len(names), (relpath, [n.name for n in keep])
    return compile(ast.Module(body=keep, type_ignores=[]), relpath, "exec")


class _DS:
    """The attributes capgan.py's allocate_dataset touches on torchvision's MNIST."""

    def __init__(self, data, targets):
        self.data, self.targets = data, targets


def _run(code, data, iid, nw, nc, ns, seed):
    rd = Random()
    rd.seed(seed)
    g = {"np": np, "torch": torch, "copy": copy, "rd": rd, "num_workers": nw, "num_class": nc,
         "num_sample": ns, "datasets": [], "test_set": None, "ims": None}
    exec(code, g)
    g["allocate_dataset"](data, iid)
    return g


def capgan_case(labels, iid, nw, nc, ns, seed=20211212):
    n = len(labels)
    code = _functions("capgan.py", ["allocate_dataset"])
    ds = _DS(torch.arange(n), torch.as_tensor(labels, dtype=torch.long))
    g = _run(code, ds, iid, nw, nc, ns, seed)
    return {"test": [int(x) for x in g["test_set"]], "shards": [[int(x) for x in d.data] for d in g["datasets"]]}


def ring_case(labels, iid, nw, nc, ns, seed=20211212):
    n = len(labels)
    code = _functions("CGLGAN/2DMG/main.py", ["allocate_dataset", "del_tensor_ele"])
    data = torch.utils.data.TensorDataset(torch.arange(n, dtype=torch.float64).view(n, 1),
                                          torch.as_tensor(labels, dtype=torch.float32))
    g = _run(code, data, iid, nw, nc, ns, seed)
    return {"test": [int(x) for x in g["test_set"].view(-1)],
            "shards": [[int(x) for x in d.view(-1)] for d in g["datasets"]]}


def main():
    rs = np.random.RandomState(0)
    lab10 = rs.randint(0, 10, size=3000)
    lab8 = np.sort(rs.randint(0, 8, size=2400)).astype(np.float32)   # gmm: labels sorted (data.py:37)
    out = {"labels10": lab10.tolist(), "labels8": lab8.tolist(), "cases": []}
    for iid in (0, 1, 2):
        for nw in (10, 4):
            out["cases"].append({"variant": "capgan", "labels": "labels10", "iid": iid, "num_workers": nw,
                                 "num_class": 10, "num_sample": 100,
                                 **capgan_case(lab10, iid, nw, 10, 100)})
        out["cases"].append({"variant": "ring", "labels": "labels8", "iid": iid, "num_workers": 8, "num_class": 8,
                             "num_sample": 100, **ring_case(lab8, iid, 8, 8, 100)})
    out["meta"] = {"numpy": np.__version__, "torch": torch.__version__,
                   "generator": "tests/golden/make_partition_golden.py"}
    path = os.path.join(OUT, "partition.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
