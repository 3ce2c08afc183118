"""HBM traffic per depth map from the two rocprofv3 PMC passes of scripts/profile_round.sh.

    python scripts/pmc_traffic.py TAG   ->  profiles/pmc_traffic.json (read by bench.py)

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports half the bytes of a
16 B/lane read, so bytes_read = 2 x FETCH_SIZE; WRITE_SIZE is exact for 16 B/lane stores. Both
counters are in KiB. The passes run bench.py with --steps 2 --warmup 1 --profile-steps 0 (3
forward steps, counted by fmt_embed_kernel dispatches); traffic per depth map = sum over one
step's dispatches of the kernels behind one C-ABI entry point (the same grouping as bench.py's
HIP-event `achieved`).
"""
import csv
import json
import os
import sys
from collections import defaultdict

ENTRY_KERNELS = {
    "tmvs_warp_corr": ("warp_corr_kernel", "warp_pair_kernel", "warp_dot_kernel"),
    "tmvs_costregnet": ("conv0_kernel", "conv3d_lds_kernel", "conv3d_direct_kernel", "conv3d_s2c8_tile_kernel",
                        "conv3d_c16_kernel", "deconv3d_lds_kernel", "deconv3d_c8_kernel", "prob_kernel",
                        "prob_wta_kernel", "softmax_wta_kernel"),
}
STEP_KERNEL = "fmt_embed_kernel"  # launched exactly once per forward step


def _is(kname, n):
    return kname.startswith(n) or f"::{n}" in kname


def load(path):
    per = defaultdict(float)
    steps = 0
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        for entry, names in ENTRY_KERNELS.items():
            if any(_is(k, n) for n in names):
                per[entry] += float(r["Counter_Value"]) * 1024.0
        if _is(k, STEP_KERNEL):
            steps += 1
    return per, max(steps, 1)


def main():
    tag = sys.argv[1]
    base = os.path.join("gpurun_out", tag)
    fetch, steps_f = load(os.path.join(base, "pmc_fetch", "run_counter_collection.csv"))
    write, steps_w = load(os.path.join(base, "pmc_write", "run_counter_collection.csv"))
    out = {"_meta": {"source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes ({tag})",
                     "formula": "2*FETCH_SIZE + WRITE_SIZE (bytes), per depth map, summed over the entry's launches",
                     "steps": steps_f}}
    for entry in ENTRY_KERNELS:
        rd = 2.0 * fetch[entry] / steps_f
        wr = write[entry] / steps_w
        out[entry] = int(rd + wr)
        out["_meta"][entry] = {"read_bytes_corrected": int(rd), "write_bytes": int(wr)}
    os.makedirs("profiles", exist_ok=True)
    with open(os.path.join("profiles", "pmc_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
