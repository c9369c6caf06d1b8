"""Print the top kernels of a rocprofv3 kernel_stats.csv: python tools/kstats.py DIR [N]"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda x: -float(x["TotalDurationNs"]))
for x in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    print(f"{x['Name'][:64]:64s} {x['Calls']:>5} {float(x['AverageNs']) / 1e3:10.1f} us {float(x['TotalDurationNs']) / 1e6:9.2f} ms")
