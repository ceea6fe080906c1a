"""HBM checkpoint tier on a real GPU (flash_checkpoint/hbm_tier.py,
engine.py _hbm_only_steps / _restore_into).

Two processes share cuda:0, as a worker and its deep standby do:
  * the STANDBY hipMallocs two staging buffers and publishes their dmabuf
    IPC handles in the agent control dir;
  * the WORKER imports them, saves step 1 (complete in shm), then step 2 with
    a slowed PCIe flush (fault injection) and SIGKILLs itself once step 2's
    snapshot is stamped complete in the standby's HBM but before its shm copy
    finished;
  * the standby then restores.  "hbm": step 2 comes back bit-exact D2D from
    its own buffers (shm holds only step 1).  "stale_pid": the stamp names
    another owner -> the HBM copies are ignored and step 1 is restored from shm.
    "noncontig": a target that cannot take the D2D path refuses the HBM-only
    step on every rank and falls back to step 1 (complete in shm).
"""

import os
import signal

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _build():
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    torch.manual_seed(0)
    cfg = GPT2Config.named("gpt2-tiny")
    with torch.device("cuda"):
        model = GPT2(cfg)
    model.to(torch.bfloat16)
    flat = FlatParams(model)
    opt = FusedAdamW(flat, lr=1e-3)
    return cfg, model, opt, flat


def _sums(flat, opt):
    return [float(flat.data.double().sum()), float(opt.exp_avg.double().sum()), float(opt.master.double().sum())]


def _env(ctl, prefix, ckdir):
    os.environ.update(DWAMD_AGENT_CTL_DIR=ctl, LOCAL_RANK="0", LOCAL_WORLD_SIZE="1", DWAMD_SHM_PREFIX=prefix,
                      CKDIR=ckdir)
    for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        os.environ.pop(k, None)


def _worker(ctl, prefix, ckdir, q):
    _env(ctl, prefix, ckdir)
    os.environ["DWAMD_FAULT_FLUSH_DELAY_S"] = "30"  # step 2's shm flush never finishes
    try:
        import time

        from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
        from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer

        torch.cuda.set_device(0)
        cfg, model, opt, flat = _build()
        x = torch.randint(0, cfg.vocab_size, (2, 65), device="cuda")
        model(x[:, :-1], x[:, 1:]).backward()
        opt.step()
        flat.zero_grad()
        ck = DdpCheckpointer(ckdir)
        state = lambda: {"model": model.state_dict(), "opt": opt.state_dict()}  # noqa: E731
        os.environ["DWAMD_FAULT_FLUSH_DELAY_S"] = "0"
        assert ck.save_checkpoint(1, state(), storage_type=StorageType.MEMORY)
        ck.wait_latest_checkpoint()
        torch.cuda.synchronize()
        s1 = _sums(flat, opt)
        cp = ck.engine._copier
        imported = bool(cp._ext) and not cp._ext[0].owned
        opt.exp_avg.add_(1.0)
        flat.data.mul_(0.5)
        torch.cuda.synchronize()
        s2 = _sums(flat, opt)
        os.environ["DWAMD_FAULT_FLUSH_DELAY_S"] = "30"
        assert ck.save_checkpoint(2, state(), storage_type=StorageType.MEMORY)
        h = ck.engine._shm_handler
        deadline = time.time() + 60
        while time.time() < deadline and not any(h.hbm_stamp(0, b)[0] == 2 for b in range(2)):
            time.sleep(0.005)
        stamped = any(h.hbm_stamp(0, b)[0] == 2 for b in range(2))
        q.put(("worker", {"s1": s1, "s2": s2, "imported": imported, "stamped": stamped,
                          "complete": sorted(h.complete_steps())}))
        time.sleep(0.5)
        os.kill(os.getpid(), signal.SIGKILL)  # mid-flush: step 2 only in the standby's HBM
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put(("worker", repr(e)))


def _standby(ctl, prefix, ckdir, q, go, mode):
    _env(ctl, prefix, ckdir)
    try:
        from dlrover_wuqiong_amd.flash_checkpoint import hbm_tier

        torch.cuda.set_device(0)
        # the payload of gpt2-tiny + AdamW state is far below 256 MiB
        ok = hbm_tier.publish_standby_buffers(ctl, 0, 256 << 20, reserve=0)
        cfg, model, opt, flat = _build()  # like a deep standby: model + optimizer already on the GPU
        q.put(("standby_ready", ok))
        if go.get(timeout=300) != "restore":
            return
        from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer

        flat.data.zero_()
        opt.exp_avg.zero_()
        opt.master.zero_()
        ck = DdpCheckpointer(ckdir)
        h = ck.engine._shm_handler
        h.init_shared_memory(create=False)
        complete_before = sorted(h.complete_steps())
        if mode == "stale_pid":
            for b in range(2):
                st, pid, nb = h.hbm_stamp(0, b)
                if st > 0:
                    h.set_hbm_stamp(0, b, st, pid + 100000, nb)  # some other (dead) owner
        state = {"model": model.state_dict(), "opt": opt.state_dict()}
        if mode == "noncontig":
            # one GPU-saved tensor restored into a non-contiguous view: cannot
            # take the D2D path of an HBM-only step
            name = next(k for k, v in state["model"].items() if v.dim() == 2)
            w = state["model"][name]
            state["model"][name] = torch.empty(w.shape[1], w.shape[0], dtype=w.dtype, device="cuda").t()
        out = ck.load_checkpoint(target=state)
        torch.cuda.synchronize()
        q.put(("standby", {"ok": ok, "sums": _sums(flat, opt),
                           "source": ck.engine.last_restore_source, "complete_before": complete_before,
                           "got": bool(out)}))
        ck.close()
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put(("standby", repr(e)))


@pytest.mark.parametrize("mode", ["hbm", "stale_pid", "noncontig"])
def test_gpu_hbm_tier_restore_after_worker_sigkill(tmp_path, _isolated_shm, mode):
    import torch.multiprocessing as mp

    ctl = str(tmp_path / "ctl")
    os.makedirs(ctl)
    ckdir = str(tmp_path / "ck")
    ctx = mp.get_context("spawn")
    q, go = ctx.Queue(), ctx.Queue()
    sb = ctx.Process(target=_standby, args=(ctl, _isolated_shm, ckdir, q, go, mode))
    sb.start()
    try:
        tag, ok = q.get(timeout=180)
        assert tag == "standby_ready" and ok is True, (tag, ok)
        wk = ctx.Process(target=_worker, args=(ctl, _isolated_shm, ckdir, q))
        wk.start()
        tag, w = q.get(timeout=180)
        assert tag == "worker" and isinstance(w, dict), w
        wk.join(timeout=60)
        assert wk.exitcode == -signal.SIGKILL, wk.exitcode
        assert w["imported"] and w["stamped"], w
        assert w["complete"] == [1], w  # step 2 never reached shm
        go.put("restore")
        tag, s = q.get(timeout=180)
        assert tag == "standby" and isinstance(s, dict), s
    finally:
        go.put("stop")
        sb.join(timeout=60)
        if sb.is_alive():
            sb.kill()
    assert s["complete_before"] == [1], s
    if mode == "hbm":
        assert s["source"] == "hbm" and s["sums"] == w["s2"], (s, w)
    elif mode == "stale_pid":
        # no stamp names this process: every byte of step 1 from shm
        assert s["source"] == "shm" and s["sums"] == w["s1"], (s, w)
    else:
        # step 2 refused on the D2D path -> step 1 (its staging buffer is
        # still stamped for this process, so it may come from HBM)
        assert s["sums"][1:] == w["s1"][1:], (s, w)
