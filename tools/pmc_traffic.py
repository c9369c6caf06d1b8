"""Per-kernel HBM traffic per launch from rocprofv3 PMC passes (tools/profile_round.sh).

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived L2 memory-side counters in KiB per dispatch.
Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports half the bytes of
wide coalesced reads, so it is doubled; WRITE_SIZE is taken as is.  Infinity-Cache hits are
counted by these counters, so the figure is L2-miss traffic (an upper bound on HBM bytes).

usage: python tools/pmc_traffic.py gpurun_out/round_TAG [out.json] [workload] [faces_per_launch]
The summary records bench.source_digest() of the tree it was run from: bench.py quotes `traffic`
only from a summary whose digest matches the code being benchmarked.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(path, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter:
                    vals[row["Kernel_Name"]].append(float(row["Counter_Value"]) * 1024.0)
    return vals


def main():
    root = sys.argv[1]
    fetch = load(os.path.join(root, "pmc_FETCH_SIZE"), "FETCH_SIZE")
    write = load(os.path.join(root, "pmc_WRITE_SIZE"), "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith(("ffd::", "void ffd::")):
            continue
        f = fetch.get(k, [])
        w = write.get(k, [])
        fr = sum(f) / len(f) if f else None
        fb = 2.0 * fr if f else None
        wb = sum(w) / len(w) if w else None
        out[k] = {"fetch_bytes": fb, "fetch_bytes_raw": fr, "write_bytes": wb, "launches": max(len(f), len(w)),
                  "traffic_bytes": (fb or 0.0) + (wb or 0.0),
                  "traffic_bytes_uncorrected": (fr or 0.0) + (wb or 0.0)}
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from bench import source_digest
    workload = sys.argv[3] if len(sys.argv) > 3 else "c2"
    per_launch = int(sys.argv[4]) if len(sys.argv) > 4 else 4096
    dg = os.path.join(root, "source_digest.txt")  # written on the GPU box by profile_round.sh
    digest = open(dg).read().strip() if os.path.exists(dg) else source_digest()
    text = json.dumps({"source": root, "source_digest": digest, "workload": workload,
                       "faces_per_launch": per_launch,
                       "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE x1; KiB -> bytes",
                       "correction_note": ("the guide states the x2 FETCH_SIZE correction for wide coalesced streaming "
                                           "reads; kernels whose reads are mostly gathers (k_traverse's 16-B node records "
                                           "beside its 16-B window staging chunks, k_votes' 32-B leaf records, "
                                           "k_meanshift's 8-B votes) may be over-stated by it: their true HBM bytes lie "
                                           "between traffic_bytes_uncorrected and traffic_bytes"),
                       "kernels": out}, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
