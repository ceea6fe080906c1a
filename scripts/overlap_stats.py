"""How much of a kernel's time ran concurrently with other kernels, from a
rocprofv3 kernel trace CSV (``rocprofv3 --kernel-trace --output-format csv``):
for every kernel whose name contains FILTER, the part of its [start, end)
covered by any kernel NOT matching the filter (e.g. the optimizer update of
optimizers/in_backward.py under the backward GEMMs).

    python scripts/overlap_stats.py run_kernel_trace.csv mt_step_kernel [--skip-first N]
Prints one JSON line: calls, total ms, overlapped ms / %, and the same for
the step window (first match to last match)."""
import csv
import json
import sys


def main():
    path, flt = sys.argv[1], sys.argv[2]
    skip = int(sys.argv[sys.argv.index("--skip-first") + 1]) if "--skip-first" in sys.argv else 0
    rows = list(csv.DictReader(open(path)))
    name_k = next(k for k in rows[0] if k.lower() in ("kernel_name", "name"))
    s_k = next(k for k in rows[0] if k.lower().startswith("start"))
    e_k = next(k for k in rows[0] if k.lower().startswith("end"))
    ks = sorted((int(r[s_k]), int(r[e_k]), r[name_k]) for r in rows)
    mine = [(s, e) for s, e, n in ks if flt in n][skip:]
    other = [(s, e) for s, e, n in ks if flt not in n]
    # merged busy intervals of the other kernels
    merged = []
    for s, e in other:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    import bisect

    starts = [m[0] for m in merged]
    tot = ov = 0
    for s, e in mine:
        tot += e - s
        i = max(0, bisect.bisect_right(starts, s) - 1)
        while i < len(merged) and merged[i][0] < e:
            a, b = max(s, merged[i][0]), min(e, merged[i][1])
            if b > a:
                ov += b - a
            i += 1
    print(json.dumps({"filter": flt, "calls": len(mine), "total_ms": round(tot / 1e6, 3),
                      "overlapped_ms": round(ov / 1e6, 3), "overlapped_pct": round(100 * ov / max(1, tot), 1),
                      "serial_ms": round((tot - ov) / 1e6, 3)}))


if __name__ == "__main__":
    main()
