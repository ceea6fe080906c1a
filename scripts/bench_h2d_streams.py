"""Pinned host -> HBM copy rate with the bytes split over 1, 2 or 4 HIP
streams (does a restore's PCIe H2D gain from more DMA queues?)."""
import json
import time

import torch


def main():
    n = 8 << 30
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    host.fill_(1)
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    for k in (1, 2, 4, 1, 2, 4):
        streams = [torch.cuda.Stream() for _ in range(k)]
        per = n // k
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                dev[i * per:(i + 1) * per].copy_(host[i * per:(i + 1) * per], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"streams": k, "GB": n / 1e9, "sec": round(dt, 4), "GBps": round(n / dt / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
