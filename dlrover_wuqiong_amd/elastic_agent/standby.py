"""Warm standby worker: a pre-started interpreter that becomes a worker.

Restarting a worker after a fault costs a fresh ``python`` + ``import torch``
(1-2 s, more on a cold page cache) before the training script even starts.
The agent therefore keeps one *standby* interpreter per local rank that has
already imported torch and this package (nothing that touches the GPU: HIP is
initialised only after the worker environment is applied) and blocks on its
stdin.  On (re)start the agent sends one JSON line -- worker environment,
argv, entrypoint, log file -- and the standby turns into the worker in
place (``runpy``, ``__main__`` semantics).  No ``exec``: the process simply
continues as the worker, so nothing GPU-initialised is ever replaced.

The reference (torchelastic-based agent) always cold-starts workers; this is
an MI355X-deployment goodput optimisation (see ``scripts/goodput_experiment.py``).
"""

import importlib
import json
import os
import runpy
import sys


def _preload():
    mods = os.environ.get("DWAMD_STANDBY_PRELOAD", "torch,torch.distributed,dlrover_wuqiong_amd.flash_checkpoint.ddp")
    for m in filter(None, (x.strip() for x in mods.split(","))):
        try:
            importlib.import_module(m)
        except Exception as e:  # a missing optional module must not kill the standby
            print(f"[standby] preload {m} failed: {e}", file=sys.stderr)


def _redirect(log_path: str):
    if not log_path:
        return
    os.makedirs(os.path.dirname(log_path) or ".", exist_ok=True)
    fd = os.open(log_path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    sys.stdout.flush()
    sys.stderr.flush()
    os.dup2(fd, 1)
    os.dup2(fd, 2)
    os.close(fd)


def main():
    _preload()
    line = sys.stdin.readline()
    if not line.strip():
        return 0  # agent discarded the standby
    cmd = json.loads(line)
    _redirect(cmd.get("log", ""))
    os.environ.clear()
    os.environ.update(cmd["env"])
    if cmd.get("cwd"):
        os.chdir(cmd["cwd"])
    entry = cmd["entry"]
    sys.argv = [entry] + list(cmd.get("args", []))
    if cmd.get("module"):
        runpy.run_module(entry, run_name="__main__", alter_sys=True)
    else:
        sys.path.insert(0, os.path.dirname(os.path.abspath(entry)))
        runpy.run_path(entry, run_name="__main__")
    return 0


if __name__ == "__main__":
    sys.exit(main())
