"""Print the last analyzeFace call's kernel / copy timeline from a latency_trace.sh run.
usage: python tools/lat_timeline.py gpurun_out/lat_TAG"""
import csv
import sys

d = sys.argv[1]
ev = []
for r in csv.DictReader(open(f"{d}/trace/run_kernel_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:48], r["Queue_Id"]))
for r in csv.DictReader(open(f"{d}/trace/run_memory_copy_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r["Direction"], "-"))
ev.sort()
idx = [i for i, e in enumerate(ev) if "gray_resize" in e[2]]
st, en = idx[-2], idx[-1]
t0 = ev[st][0]
for e in ev[st - 3:en]:
    print(f"{(e[0] - t0) / 1e3:9.1f} {(e[1] - t0) / 1e3:9.1f} {(e[1] - e[0]) / 1e3:8.1f}  q{e[3]} {e[2]}")
