"""Summarise a rocprofv3 --kernel-trace --stats CSV into markdown (for profiles/)."""

import csv
import sys


def main(stats_csv, out_md, title, steps=0):
    rows = list(csv.DictReader(open(stats_csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"# {title}", "", f"Total kernel time: {tot / 1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} dispatches"
             + (f" in {steps} steps = **{tot / 1e6 / steps:.1f} ms of kernels per step**" if steps else ""), "",
             "| kernel | calls | total ms | avg us | % |" + (" ms/step |" if steps else ""),
             "|---|---|---|---|---|" + ("---|" if steps else "")]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
        name = r["Name"].replace("|", "/")
        if len(name) > 90:
            name = name[:90] + "..."
        lines.append(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |"
                     + (f" {float(r['TotalDurationNs']) / 1e6 / steps:.2f} |" if steps else ""))
    open(out_md, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:20]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "rocprofv3 kernel stats",
         int(sys.argv[4]) if len(sys.argv) > 4 else 0)
