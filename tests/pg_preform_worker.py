"""Worker script of tests/test_pg_preform.py (run under dwamd-run, gloo).

Incarnation 0 of a single-node world waits until this node's standbys have
pre-formed their group (``standby_pg.*`` marks in the agent's control dir),
then either the last rank SIGKILLs itself (``--kill``) or every rank waits
for the agent to stop it (membership change).  Every incarnation appends
one JSON record per rank: world, rank, whether init_process_group adopted
the pre-formed group, and an all-reduce result that proves the group works.
"""

import argparse
import json
import os
import signal
import sys
import time

import torch
import torch.distributed as dist
import torch.distributed.distributed_c10d as c10d
from torch.distributed import init_process_group as imported_init  # bound before a deep standby parks

from dlrover_wuqiong_amd.elastic_agent import pg_preform


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--out", required=True)
    p.add_argument("--kill", action="store_true")
    p.add_argument("--first-world", type=int, default=0, help="world size of the incarnation that waits")
    p.add_argument("--deep", action="store_true", help="deep-standby script: parks in standby_point()")
    p.add_argument("--backend", default="gloo")
    a = p.parse_args()
    if a.deep:
        from dlrover_wuqiong_amd.elastic_agent.standby import standby_point

        standby_point(prepin_shm=False)
    t0 = time.time()
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    if not a.deep:
        dist.init_process_group(a.backend)
    elif lr % 2 == 0:
        imported_init(a.backend)  # the module-global alias taken before the standby parked
    else:
        c10d.init_process_group(a.backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t)
    inc = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
    rec = {"inc": inc, "rank": rank, "world": world, "adopted": pg_preform.adopted() is not None,
           # the patch and every rebound alias are gone after the call
           "clean": pg_preform._orig_init is None and imported_init is c10d.init_process_group is dist.init_process_group,
           "sum": float(t.item()), "init_sec": round(time.time() - t0, 4), "pid": os.getpid()}
    with open(a.out, "a") as f:
        f.write(json.dumps(rec) + "\n")
    first = (inc == 0) if a.kill else (world == a.first_world)
    if first:
        ctl = os.environ["DWAMD_AGENT_CTL_DIR"]
        lws = int(os.environ["LOCAL_WORLD_SIZE"])
        deadline = time.time() + 120
        while time.time() < deadline:
            if sum(1 for n in os.listdir(ctl) if n.startswith(pg_preform.PG_MARK_PREFIX) and not n.endswith(".tmp")) \
                    >= lws:
                break
            time.sleep(0.05)
        with open(a.out + f".ready{rank}", "w") as f:
            f.write("1")
        if a.kill and rank == world - 1:
            # every rank's record is on disk before the kill (the agent stops
            # the survivors within milliseconds of it)
            deadline = time.time() + 60
            while time.time() < deadline and sum(1 for r in range(world)
                                                 if os.path.exists(a.out + f".ready{r}")) < world:
                time.sleep(0.05)
            os.kill(os.getpid(), signal.SIGKILL)
        while True:  # stopped by the agent (failure of a peer / membership change)
            time.sleep(0.1)
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
