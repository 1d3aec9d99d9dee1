"""Prints one batch's kernel timeline (us from the batch's k_hot_precheck start) from a rocprofv3
kernel-trace CSV: python3 tools/timeline.py trace.csv [batch index from the end, default 2]."""
import csv, re, sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows:  # demangled names: keep the function name
    m = re.search(r"(k_\w+(<[^>]*>)?)\(", r["Kernel_Name"])
    if m:
        r["Kernel_Name"] = m.group(1)
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("k_hot_precheck")]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
a, b = starts[-k], starts[-k + 1] if k > 1 else len(rows)
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:b + 1]:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{s:8.1f} {e:8.1f} {e - s:7.1f}  q{r['Queue_Id']:>2}  {r['Kernel_Name'][:60]}")
