"""Side-by-side per-op ms of two bench --profile-ops files: python scripts/cmp_ops.py a.json b.json [prefix ...]"""
import json
import sys

a = json.load(open(sys.argv[1]))["op_ms"]
b = json.load(open(sys.argv[2]))["op_ms"]
pre = sys.argv[3:] or [""]
for k in a:
    if any(k.startswith(p) for p in pre):
        print(f"{k:24s} {a[k] * 1e3:8.1f} {b.get(k, float('nan')) * 1e3:8.1f}")
print(f"{'total':24s} {sum(a.values()) * 1e3:8.1f} {sum(b.values()) * 1e3:8.1f}")
