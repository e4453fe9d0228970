"""Summarise scripts/pmc_stall.sh's passes: per kernel (full template name), every counter summed
over its launches, and the ratios that say where the waves' time goes (MI355X_MICROARCH.md,
rocprofv3 PMC slots: SQ_WAIT_ANY = parked on s_waitcnt / barrier, SQ_WAIT_INST_ANY = issue
stalls, SQ_ACTIVE_INST_ANY = issuing; the three add up to SQ_WAVE_CYCLES; the SQ cycle counters
count quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES cycles; SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE =
the extra LDS cycles spent on bank conflicts)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(d):
    per = defaultdict(lambda: defaultdict(float))
    launches = defaultdict(set)
    for fn in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                k = row["Kernel_Name"]
                per[k][row["Counter_Name"]] += float(row["Counter_Value"])
                launches[k].add((os.path.dirname(fn), row.get("Dispatch_Id")))
    out = {}
    for k, c in per.items():
        r = dict(c)
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        if wc > 0:
            for key in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                        "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM",
                        "SQ_WAIT_INST_VMEM"):
                if key in c:
                    r["frac_" + key] = round(c[key] / wc, 4)
        if c.get("SQ_LDS_IDX_ACTIVE", 0) > 0 and "SQ_LDS_BANK_CONFLICT" in c:
            r["lds_conflict_frac"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 4)
        if c.get("GRBM_GUI_ACTIVE", 0) > 0 and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            r["mfma_busy_frac"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] /
                                        (c["GRBM_GUI_ACTIVE"] / 8.0 * 1024.0), 4)
        if c.get("SQ_WAVES", 0) > 0 and wc > 0:
            r["wave_quadcycles_avg"] = round(wc / c["SQ_WAVES"], 1)
        r["launch_records"] = len(launches[k])
        out[k] = r
    order = sorted(out, key=lambda k: -out[k].get("SQ_WAVE_CYCLES", 0.0))
    json.dump({k: out[k] for k in order}, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
