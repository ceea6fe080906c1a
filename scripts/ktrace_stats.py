"""Per-kernel count / mean / total time from a rocprofv3 SQLite (rocpd)
kernel trace (``rocprofv3 --kernel-trace -d DIR -o run``).
    python scripts/ktrace_stats.py gpurun_out/.../run_results.db [filter]"""
import collections
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    cols = [r[1] for r in db.execute("PRAGMA table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = db.execute(f"SELECT {name}, start, end FROM kernels").fetchall()
    agg = collections.defaultdict(list)
    for n, s, e in rows:
        if flt in n:
            agg[n.split("(")[0]].append((e - s) / 1e3)
    tot = sum(sum(v) for v in agg.values()) or 1
    print(f"| kernel | calls | mean us | min us | total ms | % |\n|---|---|---|---|---|---|")
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"| `{n[:90]}` | {len(v)} | {sum(v) / len(v):.1f} | {min(v):.1f} | {sum(v) / 1e3:.2f} | "
              f"{100 * sum(v) / tot:.1f} |")


if __name__ == "__main__":
    main()
