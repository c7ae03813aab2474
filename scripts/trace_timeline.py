import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last call: kernels after the last call_prologue_kernel
idx = max(i for i, r in enumerate(rows) if "call_prologue" in r["Kernel_Name"])
last = rows[idx:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{s/1e3:9.1f} {e/1e3:9.1f} {(e-s)/1e3:7.1f} q{r.get('Queue_Id','?')} {r['Kernel_Name'][:90]}")
print("span us", (int(last[-1]["End_Timestamp"]) - t0) / 1e3)
