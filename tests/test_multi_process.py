"""Native robust IPC primitives (parity: reference python/tests/test_multi_process.py)."""

import multiprocessing as mp
import os
import queue
import time

import pytest

from dlrover_wuqiong_amd.common.multi_process import SharedDict, SharedLock, SharedMemory, SharedQueue


def test_queue_fifo_and_sizes():
    q = SharedQueue("q1", create=True, maxsize=10, bytes_capacity=1 << 16)
    q2 = SharedQueue("q1")
    for i in range(10):
        q.put({"i": i, "pad": "x" * (i * 500)})
    with pytest.raises(queue.Full):
        q.put(1, timeout=0.05)
    assert q2.qsize() == 10
    assert [q2.get()["i"] for _ in range(10)] == list(range(10))
    assert q2.empty()
    with pytest.raises(queue.Empty):
        q2.get(timeout=0.05)
    # wraparound with variable sizes
    for r in range(50):
        q.put(b"y" * (r * 97 % 3000))
        assert len(q2.get()) == r * 97 % 3000
    q.unlink()


def test_lock_semantics():
    a = SharedLock("l1", create=True)
    b = SharedLock("l1")
    assert a.acquire(blocking=False)
    assert a.locked() and b.locked()
    assert not b.acquire(blocking=False)
    assert not b.acquire(blocking=True, timeout=0.1)
    a.release()
    assert b.acquire(blocking=False)
    b.release()
    a.unlink()


def _hold_and_die(name):
    lk = SharedLock(name)
    lk.acquire()
    os._exit(0)  # die while holding the lock


def test_lock_reclaimed_from_dead_holder():
    lk = SharedLock("l2", create=True)
    p = mp.get_context("fork").Process(target=_hold_and_die, args=("l2",))
    p.start()
    p.join()
    assert lk.acquire(blocking=True, timeout=3.0)
    lk.release()
    lk.unlink()


def test_lock_reclaimed_from_zombie_holder(_isolated_shm):
    """A SIGKILLed holder that is not reaped yet (a zombie: its parent, like
    the agent reaping in the background, has not waited) no longer owns the
    lock: a non-blocking acquire succeeds at once."""
    import signal
    import subprocess
    import sys

    lk = SharedLock("lz", create=True)
    code = ("import os, signal, sys; sys.path.insert(0, %r)\n"
            "from dlrover_wuqiong_amd.common.multi_process import SharedLock\n"
            "lk = SharedLock('lz'); lk.acquire(); print('held', flush=True); signal.pause()") % os.getcwd()
    p = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True)
    try:
        assert p.stdout.readline().strip() == "held"
        assert not lk.acquire(blocking=False)
        os.kill(p.pid, signal.SIGKILL)
        deadline = time.time() + 10
        while time.time() < deadline:  # wait for the zombie state, without reaping it
            with open(f"/proc/{p.pid}/stat") as f:
                if f.read().rsplit(")", 1)[1].split()[0] == "Z":
                    break
            time.sleep(0.01)
        assert lk.acquire(blocking=False)
        lk.release()
    finally:
        p.kill()
        p.wait()
        lk.unlink()


def _producer(name, n):
    q = SharedQueue(name)
    for i in range(n):
        q.put(i)


def test_queue_cross_process():
    q = SharedQueue("q3", create=True, maxsize=4)
    p = mp.get_context("fork").Process(target=_producer, args=("q3", 100))
    p.start()
    got = [q.get(timeout=10) for _ in range(100)]
    p.join()
    assert got == list(range(100))
    q.unlink()


def test_dict_and_memory():
    d = SharedDict("d1", create=True)
    d2 = SharedDict("d1")
    d.set({"a": 1, "b": [1, 2]})
    assert d2.get() == {"a": 1, "b": [1, 2]}
    v = d2.version()
    d2.update({"c": 3})
    assert d.get()["c"] == 3 and d.version() > v
    assert d.get(local=True)["c"] == 3
    d.unlink()
    m = SharedMemory("m1", create=True, size=8192)
    m.buf[100:105] = b"hello"
    m2 = SharedMemory("m1")
    assert bytes(m2.buf[100:105]) == b"hello"
    assert SharedMemory.exists("m1")
    m.unlink()
    assert not SharedMemory.exists("m1")


def test_storage_parallel_io(tmp_path):
    import ctypes

    from dlrover_wuqiong_amd.common.storage import PosixDiskStorage

    data = os.urandom(40 << 20)
    buf = ctypes.create_string_buffer(data, len(data))
    st = PosixDiskStorage()
    p = str(tmp_path / "x.bin")
    st.write_bytes(ctypes.addressof(buf), len(data), p, threads=8)
    out = ctypes.create_string_buffer(len(data))
    st.read_into(p, ctypes.addressof(out), len(data), threads=8)
    assert out.raw[: len(data)] == data
    from dlrover_wuqiong_amd._native import runtime

    assert runtime().dw_crc32c(buf, len(data), 0) == runtime().dw_crc32c(out, len(data), 0)


def test_storage_direct_write_aligned_body_and_tail(tmp_path):
    """dw_write_file's O_DIRECT mode: a page-aligned buffer whose length is
    not a page multiple, written at an aligned offset behind existing bytes
    (the persister's record layout); the body goes O_DIRECT, the tail
    buffered; an unaligned buffer falls back to buffered writes."""
    import ctypes

    import numpy as np

    from dlrover_wuqiong_amd._native import runtime

    n = (24 << 20) + 1234
    raw = np.frombuffer(os.urandom(n + 8192), dtype=np.uint8)
    a0 = (-raw.ctypes.data) % 4096
    src = raw[a0:a0 + n]
    assert src.ctypes.data % 4096 == 0
    p = str(tmp_path / "d.bin")
    head = os.urandom(8192)
    with open(p, "wb") as f:
        f.write(head)
    rt = runtime()
    assert rt.dw_write_file(p.encode(), ctypes.c_void_p(src.ctypes.data), n, 8192, 8, 2 | 4) == 0
    with open(p, "rb") as f:
        got = f.read()
    assert len(got) == 8192 + n and got[:8192] == head and got[8192:] == src.tobytes()
    # unaligned source: buffered path, same bytes
    q = str(tmp_path / "u.bin")
    src2 = raw[a0 + 1:a0 + 1 + n]
    assert rt.dw_write_file(q.encode(), ctypes.c_void_p(src2.ctypes.data), n, 0, 8, 1 | 2 | 4) == 0
    with open(q, "rb") as f:
        assert f.read() == src2.tobytes()


def _blocked_getter(name, prefix):
    import os

    os.environ["DWAMD_SHM_PREFIX"] = prefix
    from dlrover_wuqiong_amd.common.multi_process import SharedQueue

    q = SharedQueue(name, create=False)
    q.get(timeout=60)  # killed while waiting


def test_queue_survives_killed_waiter(_isolated_shm):
    """A waiter SIGKILLed inside get() must not wedge later put/get calls
    (process-shared condvars can; the futex-based waits cannot)."""
    import multiprocessing as mp
    import os
    import signal
    import time

    from dlrover_wuqiong_amd.common.multi_process import SharedQueue

    q = SharedQueue("kq", create=True, maxsize=4)
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_blocked_getter, args=("kq", _isolated_shm)) for _ in range(2)]
    for p in ps:
        p.start()
    time.sleep(1.5)
    for p in ps:
        os.kill(p.pid, signal.SIGKILL)
        p.join()
    t0 = time.time()
    q.put({"x": 1}, timeout=5)
    assert q.get(timeout=5) == {"x": 1}
    assert time.time() - t0 < 2.0
