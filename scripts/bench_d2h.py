"""Micro-benchmark: device->pinned-shm flush bandwidth and its interference
with concurrent GEMMs, for the copy strategies the flash-checkpoint copier can
use.  Results feed the choice in flash_checkpoint/copier.py."""

import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DWAMD_SHM_PREFIX", f"d2h{os.getpid()}")
from dlrover_wuqiong_amd._native import kernels  # noqa: E402
from dlrover_wuqiong_amd.common.multi_process import SharedMemory  # noqa: E402

GB = 1 << 30
L = kernels()
n = int(os.environ.get("D2H_GB", "8")) * GB
seg = SharedMemory("d2hbench", create=True, size=n)
t0 = time.time()
seg.prefault(16)
t_pf = time.time() - t0
t0 = time.time()
assert L.dw_host_register(ctypes.c_void_p(seg.addr), n) == 0
t_reg = time.time() - t0
dev = torch.empty(n, dtype=torch.uint8, device="cuda")
dev.random_()
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
out = {"bytes": n, "prefault_s": round(t_pf, 3), "register_s": round(t_reg, 3)}


def gemms(k=60):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(k):
        torch.matmul(a, b)
    torch.cuda.synchronize()
    return time.perf_counter() - t


gemms(10)  # warm up hipBLASLt
out["gemm_alone_s"] = round(gemms(), 4)


def run_copy(kind, stream, **kw):
    s_ptr = ctypes.c_void_p(stream.cuda_stream)
    if kind == "memcpy":
        e = L.dw_memcpy_async(ctypes.c_void_p(seg.addr), ctypes.c_void_p(dev.data_ptr()), n, 1, s_ptr)
    elif kind == "h2d":
        e = L.dw_memcpy_async(ctypes.c_void_p(dev.data_ptr()), ctypes.c_void_p(seg.addr), n, 0, s_ptr)
    else:
        dptr = L.dw_host_device_ptr(ctypes.c_void_p(seg.addr))
        e = L.dw_stream_copy(ctypes.c_void_p(dptr), ctypes.c_void_p(dev.data_ptr()), n, kw["blocks"], s_ptr)
    assert e == 0, e


def measure(name, kind, stream, **kw):
    # alone
    torch.cuda.synchronize()
    t = time.perf_counter()
    run_copy(kind, stream, **kw)
    stream.synchronize()
    alone = time.perf_counter() - t
    # concurrent with GEMMs on the default stream
    torch.cuda.synchronize()
    t = time.perf_counter()
    run_copy(kind, stream, **kw)
    g = gemms()
    stream.synchronize()
    both = time.perf_counter() - t
    out[name] = {"copy_GBps_alone": round(n / alone / 1e9, 1), "gemm_s_concurrent": round(g, 4),
                 "gemm_slowdown": round(g / out["gemm_alone_s"], 3), "total_s": round(both, 3)}


plain = torch.cuda.Stream()
measure("memcpy_plain_stream", "memcpy", plain)
measure("h2d_plain_stream", "h2d", plain)
for stride in (8, 16):
    ncu = ctypes.c_int(0)
    sp = L.dw_stream_create_cumask(stride, ctypes.byref(ncu))
    if sp:
        ext = torch.cuda.ExternalStream(sp)
        measure(f"memcpy_cumask_{ncu.value}cu", "memcpy", ext)
        measure(f"h2d_cumask_{ncu.value}cu", "h2d", ext)
for blocks in (16, 32, 64):
    measure(f"kernel_copy_{blocks}blk", "kernel", plain, blocks=blocks)
L.dw_host_unregister(ctypes.c_void_p(seg.addr))
# pageable (unregistered) H2D / D2H bandwidth
for kind, k in (("h2d_pageable", 0), ("d2h_pageable", 1)):
    torch.cuda.synchronize()
    t = time.perf_counter()
    if k == 0:
        e = L.dw_memcpy_async(ctypes.c_void_p(dev.data_ptr()), ctypes.c_void_p(seg.addr), n, 0,
                              ctypes.c_void_p(plain.cuda_stream))
    else:
        e = L.dw_memcpy_async(ctypes.c_void_p(seg.addr), ctypes.c_void_p(dev.data_ptr()), n, 1,
                              ctypes.c_void_p(plain.cuda_stream))
    L.dw_stream_sync(ctypes.c_void_p(plain.cuda_stream))
    out[kind + "_GBps"] = round(n / (time.perf_counter() - t) / 1e9, 1)
# registration with T threads over disjoint chunks
from concurrent.futures import ThreadPoolExecutor  # noqa: E402

for T in (1, 4, 8):
    chunk = n // (4 * T) // 4096 * 4096
    ranges = [(seg.addr + i * chunk, chunk) for i in range(n // chunk)]
    t = time.perf_counter()
    with ThreadPoolExecutor(T) as ex:
        rs = list(ex.map(lambda r: L.dw_host_register(ctypes.c_void_p(r[0]), r[1]), ranges))
    dt = time.perf_counter() - t
    out[f"register_{T}thr_GBps"] = round(n / dt / 1e9, 1)
    assert all(x == 0 for x in rs), rs
    for a, _ in ranges:
        L.dw_host_unregister(ctypes.c_void_p(a))

# fresh (never registered) segments: one-shot vs chunked+threaded registration
def fresh_reg(tag, chunk_mb, threads):
    s2 = SharedMemory(f"d2hfresh{tag}", create=True, size=n)
    s2.prefault(16)
    chunk = chunk_mb << 20
    ranges = [(s2.addr + o, min(chunk, n - o)) for o in range(0, n, chunk)]
    t = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        rs = list(ex.map(lambda r: L.dw_host_register(ctypes.c_void_p(r[0]), r[1]), ranges))
    dt = time.perf_counter() - t
    assert all(x == 0 for x in rs)
    # H2D from it to check the registration is effective
    torch.cuda.synchronize()
    t = time.perf_counter()
    for a, b in ranges:
        L.dw_memcpy_async(ctypes.c_void_p(dev.data_ptr() + (a - s2.addr)), ctypes.c_void_p(a), b, 0,
                          ctypes.c_void_p(plain.cuda_stream))
    L.dw_stream_sync(ctypes.c_void_p(plain.cuda_stream))
    h2d = n / (time.perf_counter() - t) / 1e9
    for a, _ in ranges:
        L.dw_host_unregister(ctypes.c_void_p(a))
    s2.unlink()
    out[f"fresh_register_{chunk_mb}MB_{threads}thr"] = {"GBps": round(n / dt / 1e9, 1), "h2d_GBps": round(h2d, 1)}


fresh_reg("a", n >> 20, 1)
fresh_reg("b", 256, 1)
fresh_reg("c", 256, 8)
print(json.dumps(out))
del dev
seg.unlink()
