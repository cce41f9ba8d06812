"""Per-step kernel statistics from a rocprofv3 kernel-trace CSV of scripts/train_trace.py: the
dispatches between the two marker kernels (torch.cuda._sleep), divided by the step count.

    python scripts/trace_steps.py TRACE.csv STEPS OUT.csv
"""
import csv
import sys
from collections import defaultdict


def main():
    path, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"] or "sleep" in r["Kernel_Name"].lower()]
    assert len(marks) >= 2, marks
    lo, hi = marks[-2], marks[-1]
    agg = defaultdict(lambda: [0, 0])
    for r in rows[lo + 1:hi]:
        a = agg[r["Kernel_Name"]]
        a[0] += 1
        a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    span = (int(rows[hi]["Start_Timestamp"]) - int(rows[lo]["End_Timestamp"])) / 1e6 / steps
    busy = sum(v[1] for v in agg.values()) / 1e6 / steps
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "CallsPerStep", "MsPerStep", "AvgUs"])
        for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            w.writerow([k, round(n / steps, 2), round(t / 1e6 / steps, 4), round(t / n / 1e3, 2)])
    print(f"wall {span:.2f} ms/step, kernel time {busy:.2f} ms/step, {sum(v[0] for v in agg.values()) / steps:.0f} "
          f"dispatches/step")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"{t / 1e6 / steps:8.3f} ms {n / steps:7.1f}x  {k[:110]}")


if __name__ == "__main__":
    main()
