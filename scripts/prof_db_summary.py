"""Summarise a rocprofv3 SQLite (rocpd) kernel trace: per-kernel time over
the last ``--steps`` training steps (steps found from the periodic adam
kernel), as a markdown table."""
import argparse
import collections
import sqlite3


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--marker", default="adam_flat_kernel", help="kernel launched once per step")
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--top", type=int, default=40)
    a = p.parse_args()
    con = sqlite3.connect(a.db)
    cur = con.cursor()
    names = {kid: (dn or kn) for kid, kn, dn in cur.execute(
        "select id, kernel_name, display_name from rocpd_info_kernel_symbol")}
    rows = list(cur.execute("select kernel_id, start, end, grid_size_x, grid_size_y, grid_size_z, "
                            "workgroup_size_x from rocpd_kernel_dispatch order by start"))
    marks = [r[1] for r in rows if a.marker in names[r[0]]]
    t0 = marks[-a.steps - 1] if len(marks) > a.steps else rows[0][1]
    t1 = marks[-1]
    win = [r for r in rows if t0 < r[1] <= t1]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for kid, s, e, *_ in win:
        agg[names[kid]][0] += 1
        agg[names[kid]][1] += (e - s) / 1e6
    total = sum(v[1] for v in agg.values())
    wall = (t1 - t0) / 1e6
    print(f"Steady state: {a.steps} steps, wall {wall / a.steps:.2f} ms/step, kernel busy "
          f"{total / a.steps:.2f} ms/step ({100 * total / wall:.1f} %)\n")
    print("| kernel | calls/step | ms/step | avg us | % |\n|---|---|---|---|---|")
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        short = n if len(n) < 90 else n[:87] + "..."
        print(f"| `{short}` | {c / a.steps:.0f} | {t / a.steps:.3f} | {1000 * t / c:.1f} | {100 * t / total:.1f} |")


if __name__ == "__main__":
    main()
