"""Summarise scripts/pmc_kernel.sh output: per (kernel, grid) mean counter values + derived ratios.

    python scripts/pmc_report.py TAG [name-filter]
"""
import collections
import csv
import glob
import re
import sys

tag = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob(f"gpurun_out/{tag}/pmc_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        name = re.sub(r"^void tmvs::|\(.*$", "", r["Kernel_Name"])[:60]
        if filt and filt not in name:
            continue
        vals[(name, int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (name, grid), d in sorted(vals.items(), key=lambda x: (x[0][0], x[0][1])):
    m = {k: sum(v) / len(v) for k, v in d.items()}
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8  # per XCD
    line = [f"{name:60s} grid={grid:>9d}", f"us={cyc / 2400:7.1f}" if cyc else ""]
    if cyc and "TA_TA_BUSY_sum" in m:
        line.append(f"TA={m['TA_TA_BUSY_sum'] / 256 / cyc:5.2f}")
    if cyc and "SQ_INSTS_VALU" in m:
        line.append(f"VALU={m['SQ_INSTS_VALU'] * 2 / 1024 / cyc:5.2f}")
    if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        line.append(f"MFMA={m['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / cyc:5.2f}")
    if "FETCH_SIZE" in m:
        line.append(f"rdMB={2 * m['FETCH_SIZE'] / 1024:8.1f}")
    if "WRITE_SIZE" in m:
        line.append(f"wrMB={m['WRITE_SIZE'] / 1024:8.1f}")
    if cyc and "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        gbs = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024 / (cyc / 2.4e9) / 1e9
        line.append(f"GB/s={gbs:7.0f}")
    if "SQ_LDS_IDX_ACTIVE" in m and m["SQ_LDS_IDX_ACTIVE"]:
        line.append(f"ldsconf={m.get('SQ_LDS_BANK_CONFLICT', 0) / m['SQ_LDS_IDX_ACTIVE']:4.2f}")
    if cyc and "TA_ADDR_STALLED_BY_TC_CYCLES_sum" in m:
        line.append(f"TAstallTC={m['TA_ADDR_STALLED_BY_TC_CYCLES_sum'] / 256 / cyc:4.2f}")
    if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
        line.append(f"L2hit={m['TCC_HIT_sum'] / max(m['TCC_HIT_sum'] + m['TCC_MISS_sum'], 1):4.2f}")
    if "TCP_TOTAL_CACHE_ACCESSES_sum" in m and "TCP_TCC_READ_REQ_sum" in m:
        line.append(f"L1miss={m['TCP_TCC_READ_REQ_sum'] / max(m['TCP_TOTAL_CACHE_ACCESSES_sum'], 1):4.2f}")
    if cyc and "SQ_WAIT_ANY" in m and "SQ_WAVE_CYCLES" in m:
        line.append(f"parked={m['SQ_WAIT_ANY'] / max(m['SQ_WAVE_CYCLES'], 1):4.2f}")
    if "SQ_WAVE_CYCLES" in m and cyc:  # SQ_WAVE_CYCLES counts quad-cycles (MI355X_MICROARCH.md)
        line.append(f"waves/SIMD={4 * m['SQ_WAVE_CYCLES'] / 1024 / cyc:4.1f}")
    if cyc and "SQ_WAIT_INST_ANY" in m and "SQ_WAVE_CYCLES" in m:
        line.append(f"wait={m['SQ_WAIT_INST_ANY'] / max(m['SQ_WAVE_CYCLES'], 1):4.2f}")
    print(" ".join(x for x in line if x))
