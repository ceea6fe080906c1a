"""GPU trace analysis: kernel time by category and how much collective
(RCCL) time is hidden behind compute.

Inputs: a torch.profiler Chrome trace (``prof.export_chrome_trace``; GPU
kernels are the ``"cat": "kernel"`` complete events) or a ``rocprofv3
--kernel-trace --output-format csv`` kernel trace (``Kernel_Name``,
``Start_Timestamp``, ``End_Timestamp`` in ns).

``analyze(kernels)`` returns:
  * per-category busy time (gemm / attention / communication / norm /
    elementwise / optimizer / copy / other) and the top kernels;
  * ``comm_s``: union of collective-kernel intervals; ``exposed_comm_s``:
    the part of it with no compute kernel running -- the time a better
    bucket / stream overlap could still win; ``overlap_pct``.

``python -m dlrover_wuqiong_amd.utils.trace_analysis trace.json|kernel_trace.csv``

Parity: ATorch ``atorch/utils/parse_trace_json.py`` (analyze_gpu_kernel,
analyze_communicate_overlap).
"""

import csv
import json
import re
import sys
from collections import defaultdict
from typing import Dict, List, Tuple

Kernel = Tuple[str, float, float]  # name, start_s, end_s

_CATS = [
    ("communication", re.compile(r"nccl|rccl|AllReduce|AllGather|ReduceScatter|AllToAll|Broadcast|SendRecv", re.I)),
    ("attention", re.compile(r"attn|flash|fmha|sdpa|softmax", re.I)),
    ("gemm", re.compile(r"Cijk_|gemm|gemv|matmul|mfma|hipblaslt|rocblas|grouped_gemm", re.I)),
    ("optimizer", re.compile(r"adam|agd|multi_tensor_apply|sgd|lamb", re.I)),
    ("norm", re.compile(r"norm", re.I)),
    ("copy", re.compile(r"copy|memcpy|memset|fill", re.I)),
    ("elementwise", re.compile(r"elementwise|gelu|silu|swiglu|rope|colred|xent|reduce|vectorized", re.I)),
]


def category(name: str) -> str:
    for cat, rx in _CATS:
        if rx.search(name):
            return cat
    return "other"


def load_chrome_trace(path: str) -> List[Kernel]:
    with open(path) as f:
        obj = json.load(f)
    events = obj["traceEvents"] if isinstance(obj, dict) else obj
    out = []
    for e in events:
        if e.get("ph") == "X" and e.get("cat") in ("kernel", "gpu_memcpy", "gpu_memset"):
            ts = float(e["ts"]) * 1e-6
            out.append((e.get("name", "?"), ts, ts + float(e.get("dur", 0)) * 1e-6))
    return out


def load_rocprof_csv(path: str) -> List[Kernel]:
    out = []
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            out.append((row["Kernel_Name"], int(row["Start_Timestamp"]) * 1e-9, int(row["End_Timestamp"]) * 1e-9))
    return out


def load(path: str) -> List[Kernel]:
    return load_rocprof_csv(path) if path.endswith(".csv") else load_chrome_trace(path)


def _union(iv: List[Tuple[float, float]]) -> List[Tuple[float, float]]:
    out: List[Tuple[float, float]] = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], b))
        else:
            out.append((a, b))
    return out


def _length(iv) -> float:
    return sum(b - a for a, b in iv)


def _intersect(x, y) -> float:
    i = j = 0
    tot = 0.0
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if b > a:
            tot += b - a
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return tot


def analyze(kernels: List[Kernel], top: int = 10) -> Dict:
    by_cat: Dict[str, float] = defaultdict(float)
    by_name: Dict[str, List[float]] = defaultdict(lambda: [0.0, 0])
    comm, comp = [], []
    for name, a, b in kernels:
        c = category(name)
        by_cat[c] += b - a
        by_name[name][0] += b - a
        by_name[name][1] += 1
        (comm if c == "communication" else comp).append((a, b))
    cu, pu = _union(comm), _union(comp)
    comm_s = _length(cu)
    hidden = _intersect(cu, pu)
    span = (max(b for _, _, b in kernels) - min(a for _, a, _ in kernels)) if kernels else 0.0
    busy = _length(_union(comm + comp))
    return {
        "kernels": len(kernels), "span_s": span, "busy_s": busy, "idle_s": max(0.0, span - busy),
        "by_category_s": dict(sorted(by_cat.items(), key=lambda kv: -kv[1])),
        "top_kernels": [{"name": n, "total_s": t, "calls": c}
                        for n, (t, c) in sorted(by_name.items(), key=lambda kv: -kv[1][0])[:top]],
        "comm_s": comm_s, "exposed_comm_s": comm_s - hidden,
        "overlap_pct": 100.0 * hidden / comm_s if comm_s else None,
    }


def main(argv=None):
    argv = argv if argv is not None else sys.argv[1:]
    res = analyze(load(argv[0]))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
