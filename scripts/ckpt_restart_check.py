"""Two-process check of the double-buffered flash checkpoint on the GPU.

Process A trains a few steps, saves to memory twice (slot 0, slot 1) and
exits with a save in flight (like a crash).  Process B (fresh HIP context)
restores from memory, then saves several more times into both slots, and
verifies every restore.  The parent never touches the GPU.
"""

import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(phase: str, model: str):
    sys.path.insert(0, REPO)
    import torch

    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
    from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    torch.manual_seed(0)
    cfg = GPT2Config.named(model)
    with torch.device("cuda"):
        m = GPT2(cfg)
    m.to(torch.bfloat16)
    flat = FlatParams(m)
    opt = FusedAdamW(flat, lr=1e-4)
    x = torch.randint(0, cfg.vocab_size, (2, 257), device="cuda")

    def train():
        m(x[:, :-1], x[:, 1:]).backward()
        opt.step()
        flat.zero_grad()

    def state(step):
        return {"model": m.state_dict(), "opt": opt.state_dict(), "step": step}

    ck = DdpCheckpointer("/tmp/dwamd_restart_check")
    h = ck.engine._shm_handler
    out = {"phase": phase}
    if phase == "A":
        for step in (1, 2, 3):
            train()
            ck.save_checkpoint(step, state(step), storage_type=StorageType.MEMORY)
            if step < 3:
                ck.wait_latest_checkpoint()
            torch.cuda.current_stream().synchronize()
        out["sum_after_2"] = None
        out["steps"] = h.complete_steps()
        print(json.dumps(out), flush=True)
        os._exit(17)  # step 3's flush may be in flight
    t0 = time.time()
    r = ck.load_checkpoint(target=state(0))
    torch.cuda.synchronize()
    out["restored_step"] = r.get("step") if r else None
    out["restore_s"] = round(time.time() - t0, 3)
    out["steps_at_start"] = {str(k): v for k, v in h.complete_steps().items()}
    errs = []
    for step in range(10, 16):
        train()
        torch.cuda.current_stream().synchronize()
        ref = float(flat.data.float().sum())
        try:
            ck.save_checkpoint(step, state(step), storage_type=StorageType.MEMORY)
            ck.wait_latest_checkpoint()
        except Exception as e:
            errs.append(f"step {step}: {e}")
            break
        flat.data.zero_()
        r = ck.load_checkpoint(target=state(0))
        torch.cuda.synchronize()
        got = float(flat.data.float().sum())
        if r.get("step") != step or got != ref:
            errs.append(f"step {step}: restored {r.get('step')} sum {got} != {ref}")
    out["errors"] = errs
    out["ranges"] = len(ck.engine._copier.pinned._ranges)
    out["final_steps"] = {str(k): v for k, v in h.complete_steps().items()}
    ck.close()
    print(json.dumps(out), flush=True)
    sys.exit(1 if errs else 0)


def main():
    model = sys.argv[2] if len(sys.argv) > 2 else "gpt2-medium"
    env = dict(os.environ, DWAMD_SHM_PREFIX=f"rc{os.getpid()}")
    rc = 0
    for phase in ("A", "B"):
        p = subprocess.run([sys.executable, __file__, "child", model, phase], env=env, timeout=300)
        print(f"phase {phase} rc={p.returncode}", flush=True)
        if phase == "B":
            rc = p.returncode
    import glob

    for f in glob.glob(f"/dev/shm/dwamd_rc{os.getpid()}*"):
        os.remove(f)
    return rc


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child(sys.argv[3], sys.argv[2])
    else:
        sys.exit(main())
