"""Generate PFM golden vectors from the REAL reference's datasets/data_io.py (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_io.py

Loads /root/reference/datasets/data_io.py by path. Its read_pfm/save_pfm need only numpy / re /
sys; the module also imports cv2 (absent here) for a RandomCrop class that is never used, so an
empty test-only ``cv2`` module is placed in sys.modules for the import. It then writes seeded float32 arrays through its save_pfm
(greyscale and colour) and stores the resulting file bytes + the arrays read back by its
read_pfm in tests/golden/pfm.npz. Data only: no reference source is copied.
"""
import importlib.util
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/datasets/data_io.py"


def main():
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))  # only RandomCrop (unused) needs it
    spec = importlib.util.spec_from_file_location("ref_data_io", REF)
    dio = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(dio)
    rng = np.random.Generator(np.random.PCG64(7))
    grey = (425.0 + 510.0 * rng.random((13, 17))).astype(np.float32)
    colour = rng.random((5, 7, 3)).astype(np.float32)
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for name, arr in (("grey", grey), ("colour", colour)):
            fn = os.path.join(td, name + ".pfm")
            dio.save_pfm(fn, arr.copy())
            raw = open(fn, "rb").read()
            back, scale = dio.read_pfm(fn)
            out[name + "_in"] = arr
            out[name + "_bytes"] = np.frombuffer(raw, np.uint8)
            out[name + "_read"] = np.ascontiguousarray(back)
            out[name + "_scale"] = np.float64(scale)
    np.savez_compressed(os.path.join(HERE, "pfm.npz"), **out)
    print("wrote", os.path.join(HERE, "pfm.npz"), {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
