"""Compatibility import path (reference: atorch/atorch/utils/parse_trace_json.py).

Thin re-export onto the MI355X-native implementation in ``dlrover_wuqiong_amd.utils.trace_analysis``;
existing ATorch user code imports unchanged.
"""

from dlrover_wuqiong_amd.utils.trace_analysis import analyze, load, load_chrome_trace, load_rocprof_csv, main  # noqa: F401
