"""Find walk_setup_kernel launches far above their median in a rocprofv3 kernel trace and print
their launch shape plus the kernels around them."""
import csv, statistics, sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
ws = [i for i, r in enumerate(rows) if "walk_setup" in r["Kernel_Name"]]
d = [rows[i]["e"] - rows[i]["s"] for i in ws]
med = statistics.median(d)
print("walk_setup launches", len(ws), "median us", med / 1e3, "max us", max(d) / 1e3)
keys = [k for k in rows[0] if k not in ("Kernel_Name", "s", "e")]
t0 = rows[0]["s"]
for n, (i, dur) in enumerate(zip(ws, d)):
    if dur < 20 * med:
        continue
    r = rows[i]
    print("SLOW", dur / 1e3, "us", "poll #", n, "of", len(ws), "at ms", (r["s"] - t0) / 1e6,
          "after the first kernel", {k: r[k] for k in keys if "Size" in k or "Count" in k or "Queue" in k or "Stream" in k})
    for j in range(max(0, i - 4), min(len(rows), i + 4)):
        q = rows[j]
        gap = (q["s"] - rows[j - 1]["e"]) / 1e3 if j else 0
        print("   ", j - i, q["Kernel_Name"][:50], "dur us", (q["e"] - q["s"]) / 1e3, "gap us", gap,
              "q", q.get("Queue_Id"), "grid", q.get("Grid_Size_X", q.get("Grid_Size")), "lds", q.get("LDS_Block_Size"))
