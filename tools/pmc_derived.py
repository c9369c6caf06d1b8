"""Per-kernel SQ counter totals per dispatch (summed over the counter's instances, averaged over
dispatches) from tools/pmc.sh passes, with derived ratios:
  wait_frac        = SQ_WAIT_ANY / SQ_WAVE_CYCLES             (wave-cycles spent waiting on anything)
  valu_active_frac = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES      (wave-cycles issuing VALU)
  lds_conflict     = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE  (LDS cycles lost to bank conflicts)
usage: python tools/pmc_derived.py gpurun_out/pmc_TAG out.json [kernel-substring ...]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    root, out = sys.argv[1], sys.argv[2]
    keys = sys.argv[3:]
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> dispatch -> sum
    for f in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            if keys and not any(s in k for s in keys):
                continue
            per[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    res = {}
    for k, cs in sorted(per.items()):
        c = {n: sum(d.values()) / len(d) for n, d in cs.items()}
        row = {"counters_per_dispatch": {n: round(v) for n, v in sorted(c.items())}}
        if c.get("SQ_WAVE_CYCLES"):
            if "SQ_WAIT_ANY" in c:
                row["wait_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4)
            if "SQ_ACTIVE_INST_VALU" in c:
                row["valu_active_frac"] = round(c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"], 4)
        if c.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in c:
            row["lds_conflict"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 4)
        res[k] = row
    json.dump(res, open(out, "w"), indent=1)
    for k, row in res.items():
        print(k[:60], {x: row[x] for x in ("wait_frac", "valu_active_frac", "lds_conflict") if x in row})


if __name__ == "__main__":
    main()
