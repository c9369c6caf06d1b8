"""Summarise PMC passes (tools/pmc.sh output dir) per kernel: mean counter value per dispatch.
usage: python tools/pmc_table.py gpurun_out/pmc_TAG [kernel-substring ...]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    keys = sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if keys and not any(s in k for s in keys):
                continue
            m = re.search(r"(k_\w+(?:<[^>]*>)?)", k)  # (anonymous-namespace kernels: "ffd::(anonymous namespace)::k_...")
            acc[m.group(1) if m else k.split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
