"""N>1 fault path rehearsed on ONE GPU (bench.py --rehearse-shared-device):
2 ranks share cuda:0 over gloo (RCCL refuses two ranks per device) with
2 deep standbys, per-slice HBM-tier staging, a SIGKILL of rank 1 mid-step
while the last checkpoint's shm flush is still running (fault injection),
agent restart, and a restore of the HBM-only step through the SAME branches
an RCCL world takes (each rank copies its slice D2D from its HBM buffer, the
slices meet in an all-gather -- staged through pinned host memory over gloo
-- and one kernel scatters them into the live tensors; the persisted file is
read 1/N per rank and all-gathered the same way) -- then the same failure
under the default import standbys.  Never an
N-GPU measurement: the JSON says ``rehearsal: true``."""

import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(400)
@pytest.mark.parametrize("ranks", [2, 4])
def test_gpu_rehearse_ranks_shared_device(tmp_path, ranks):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    # the rehearsal's 2-4 workers + standbys share this card with the test
    # process: hand back what earlier tests left in this process's cache
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", str(ranks), "--rehearse-shared-device",
           "--model", "gpt2", "--micro-batch", "2", "--seq", "256", "--steps", "4", "--warmup", "2",
           "--fault-window", "12", "--import-window", "8", "--inject-slow-flush", "3",
           "--ckpt-dir", str(tmp_path / "ckpt"), "--timeout", "300"]
    log = tmp_path / "bench.err"
    with open(log, "w") as err:
        r = subprocess.run(cmd, env=env, cwd=REPO, stdout=subprocess.PIPE, stderr=err, text=True, timeout=380)
    tail = log.read_text()[-20000:]
    sys.stderr.write(tail[-6000:])
    assert r.returncode == 0, tail
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    print(json.dumps(res))
    assert res["rehearsal"] is True and res["n_gpus"] == 1 and res["rccl_world"] == ranks
    assert res["backend"] == "gloo" and "rehearsal" in res["config"]["parallelism"]
    assert res["load_verified"] and res["replicas_identical"] and res["timed_saves_ok"]
    assert res["restarts"] == 1 and res["load_verified_after_restart"]
    # the killed step's checkpoint existed only in the standbys' HBM: each
    # rank copied its slice D2D, then the slices met in the all-gather
    assert res["restore_source"] == "hbm", res["restore_source"]
    g = res["restore_gather"]
    assert g["transport"] == "host-staged" and g["rounds"] >= 1, g
    assert res["load_storage_verified"] is True
    assert res["load_storage_stats"].get("gather_transport") == "host-staged", res["load_storage_stats"]
    imp = res["import_mode"]
    assert imp["restarts"] == 1 and imp["load_verified_after_restart"]
