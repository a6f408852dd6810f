"""Sum rocprofv3 --pmc counter_collection CSVs per counter over the
dispatches of one kernel (name substring), plus the derived figures used in
profiles/pmc/: MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
GRBM_GUI_ACTIVE / 8 XCDs), LDS bank-conflict and wait shares of wave cycles,
L2 hit rate.

    python scripts/pmc_summary.py KERNEL_SUBSTR file [file ...]   (rocpd .db or counter_collection .csv)
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def main():
    sub, files = sys.argv[1], sys.argv[2:]
    tot = defaultdict(float)
    disp = set()
    for f in files:
        if f.endswith(".db"):
            c = sqlite3.connect(f)
            q = ("select dispatch_id, counter_name, value from counters_collection where kernel_name like ?")
            for did, name, val in c.execute(q, (f"%{sub}%",)):
                disp.add((f, did))
                tot[name] += float(val)
            continue
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
                if sub not in name:
                    continue
                disp.add((f, row.get("Dispatch_Id") or row.get("Dispatch-Id")))
                tot[row["Counter_Name"]] += float(row["Counter_Value"])
    print(f"kernel ~ {sub}: {len(disp)} dispatches")
    for k in sorted(tot):
        print(f"{k:32s} {tot[k]:20.0f}")
    g = tot.get("GRBM_GUI_ACTIVE")
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in tot:
        print(f"MFMA busy = {tot['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * g / 8):.3f}")
    if tot.get("SQ_WAVE_CYCLES"):
        w = tot["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_LDS", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in tot:
                print(f"{k} / SQ_WAVE_CYCLES = {tot[k] / w:.3f}")
    if tot.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in tot:
        print(f"LDS bank-conflict cycles per LDS instruction = {tot['SQ_LDS_BANK_CONFLICT'] / tot['SQ_INSTS_LDS']:.3f}")
    if tot.get("TCC_HIT_sum") is not None and tot.get("TCC_MISS_sum") is not None:
        h, m = tot["TCC_HIT_sum"], tot["TCC_MISS_sum"]
        if h + m:
            print(f"L2 hit rate = {h / (h + m):.3f}")


if __name__ == "__main__":
    main()
