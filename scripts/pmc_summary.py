"""Summarise the two rocprofv3 PMC passes of scripts/pmc.sh into HBM bytes per kernel launch.

FETCH_SIZE and WRITE_SIZE are rocprofv3 derived counters in KiB (from TCC_EA0_RDREQ/_WRREQ).
MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE reports exactly half of the bytes of a
wide (16 B/lane) coalesced read, so it is doubled; WRITE_SIZE is exact for 16 B/lane stores.
Both count Infinity-Cache (L3) hits as fabric traffic, i.e. these are L2-miss bytes, an upper
bound on true HBM bytes.  Output: JSON with per-family launch counts and bytes per launch.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def family(name):
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    return re.split(r"[<(]", n, 1)[0].strip()


def read_pass(d, counter, optional=False, sub=None):
    """Per-family sum of `counter` (and launch counts) from the pass in d/<sub or counter>."""
    sub = sub or ("MFMA" if counter == "SQ_VALU_MFMA_BUSY_CYCLES" else counter)
    files = glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        if optional:
            return {}, {}
        raise SystemExit("no counter_collection.csv under %s/%s" % (d, sub))
    per = defaultdict(float)     # family -> summed counter
    launches = defaultdict(set)  # family -> dispatch ids
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                fam = family(row["Kernel_Name"])
                per[fam] += float(row["Counter_Value"])
                launches[fam].add(row["Dispatch_Id"])
    return per, {k: len(v) for k, v in launches.items()}


def lib_sha(path):
    """First 16 hex digits of the sha256 of the built library (the build stamp)."""
    import hashlib
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--steps", type=int, default=2, help="train steps covered by the passes")
    ap.add_argument("--lib", default=os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "tmrnet_amd", "libtmr.so"),
        help="the library the passes ran (its sha256 stamps the record; bench.py load_traffic "
             "drops a record whose stamp differs from the library it runs)")
    args = ap.parse_args()
    fetch, nf = read_pass(args.dir, "FETCH_SIZE")
    write, nw = read_pass(args.dir, "WRITE_SIZE")
    fams = {}
    for fam in sorted(set(fetch) | set(write)):
        n = max(nf.get(fam, 0), nw.get(fam, 0))
        rd = 2.0 * fetch.get(fam, 0.0) * 1024.0
        wr = write.get(fam, 0.0) * 1024.0
        fams[fam] = {"launches": n, "read_bytes": int(rd), "write_bytes": int(wr),
                     "hbm_bytes_per_launch": int((rd + wr) / max(1, n)),
                     "hbm_bytes_per_step": int((rd + wr) / args.steps)}
    busy, _ = read_pass(args.dir, "SQ_VALU_MFMA_BUSY_CYCLES", optional=True)
    gui, _ = read_pass(args.dir, "GRBM_GUI_ACTIVE", optional=True, sub="MFMA")
    for fam, d in fams.items():
        if fam in busy and gui.get(fam, 0) > 0:
            # busy cycles summed over all 1024 SIMDs / (kernel cycles = GUI_ACTIVE over 8 XCDs / 8)
            d["mfma_busy_frac"] = round(busy[fam] / (gui[fam] / 8.0 * 1024.0), 4)
            d["mfma_busy_cycles"] = busy[fam]
            d["gui_active_cycles"] = gui[fam]
    out = {"model": args.model, "steps": args.steps, "build_sha": lib_sha(args.lib),
           "what": "bench.py --steps 1 --warmup 1 (2 train steps + setup), rocprofv3 --pmc "
                   "FETCH_SIZE / WRITE_SIZE in separate passes, kernel-trace only",
           "correction": "read = 2 x FETCH_SIZE(KiB) x 1024 (gfx950 wide-read halving); "
                         "write = WRITE_SIZE(KiB) x 1024",
           "families": fams}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
