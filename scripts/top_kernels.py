"""Per-kernel table of a train step: time (rocprofv3 --kernel-trace --stats of scripts/profile.sh),
HBM bytes and MFMA busy (the PMC record of scripts/pmc.sh for the same library build) -- the
"per-kernel rocprof MFMA-busy % and HBM GB/s for the top kernels" of SURVEY.md §8d.

usage: python scripts/top_kernels.py <run_kernel_stats.csv> <pmc_traffic_*.json> [--top 15]

Kernels are grouped by family (the name before its template / parameter list, as
scripts/pmc_summary.py keys the PMC record); steps in the profiled run are counted by the
optimizer launch (one sgd_multi_k per step).  GB/s = the family's PMC bytes per step over its
profiled time per step (FETCH_SIZE doubled per the gfx950 correction + WRITE_SIZE: L2-miss bytes,
an upper bound on HBM bytes); MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES over the family's launches /
(GRBM_GUI_ACTIVE / 8 x 1024 SIMDs).
"""
import argparse
import csv
import json
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import family  # noqa: E402


def pretty(fam):
    """Display name: the identifier of a mangled name (templated kernels in an anonymous
    namespace keep their mangled names in the traces; the binutils demangler lacks __bf16)."""
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)", fam) or re.match(r"_Z(\d+)", fam)
    if not m:
        return fam
    n = int(m.group(1))
    return fam[m.end():m.end() + n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("pmc")
    ap.add_argument("--top", type=int, default=15)
    args = ap.parse_args()
    ns = defaultdict(float)
    calls = defaultdict(int)
    steps = 0
    with open(args.stats) as f:
        for r in csv.DictReader(f):
            fam = family(r["Name"])
            ns[fam] += float(r["TotalDurationNs"])
            calls[fam] += int(r["Calls"])
            if fam == "sgd_multi_k":
                steps += int(r["Calls"])
    if steps == 0:
        raise SystemExit("no sgd_multi_k launches: cannot count the profiled steps")
    with open(args.pmc) as f:
        pmc = json.load(f)
    fams = pmc["families"]
    tot = sum(ns.values()) / steps / 1e6
    print("library %s; %d profiled steps, %.1f ms of kernels per step" % (pmc.get("build_sha"), steps, tot))
    print()
    print("| kernel family | ms / step | share | launches / step | HBM GB/s (PMC) | MFMA busy |")
    print("|---|---|---|---|---|---|")
    for fam in sorted(ns, key=lambda k: -ns[k])[:args.top]:
        ms = ns[fam] / steps / 1e6
        p = fams.get(fam)
        gbs = "%.0f" % (p["hbm_bytes_per_step"] / (ms * 1e-3) / 1e9) if p and ms > 0 else "-"
        busy = "%.0f%%" % (100 * p["mfma_busy_frac"]) if p and p.get("mfma_busy_frac") else "-"
        print("| `%s` | %.2f | %.1f%% | %.0f | %s | %s |" % (pretty(fam), ms, 100 * ms / tot,
                                                          calls[fam] / steps, gbs, busy))


if __name__ == "__main__":
    main()
