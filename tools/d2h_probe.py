"""Achievable D2H / H2D rate on the box for frame-sized copies into pinned host memory (dev tool):
    python tools/d2h_probe.py      (one JSON line per configuration)"""
import json
import time

import torch


def main():
    fb = 3133440  # 1080p 4:2:0 frame
    n = 256
    dev = torch.empty(n * fb, dtype=torch.uint8, device="cuda:0")
    host = torch.empty(n * fb, dtype=torch.uint8, pin_memory=True)
    for nstreams in (1, 2, 4, 8):
        streams = [torch.cuda.Stream() for _ in range(nstreams)]
        for rep in range(2):
            torch.cuda.synchronize()
            t = time.perf_counter()
            for i in range(n):
                with torch.cuda.stream(streams[i % nstreams]):
                    host[i * fb:(i + 1) * fb].copy_(dev[i * fb:(i + 1) * fb], non_blocking=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
        print(json.dumps({"dir": "D2H", "streams": nstreams, "GBps": round(n * fb / dt / 1e9, 2)}))
    for nstreams in (1, 4):
        streams = [torch.cuda.Stream() for _ in range(nstreams)]
        for rep in range(2):
            torch.cuda.synchronize()
            t = time.perf_counter()
            for i in range(n):
                with torch.cuda.stream(streams[i % nstreams]):
                    dev[i * fb:(i + 1) * fb].copy_(host[i * fb:(i + 1) * fb], non_blocking=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
        print(json.dumps({"dir": "H2D", "streams": nstreams, "GBps": round(n * fb / dt / 1e9, 2)}))


if __name__ == "__main__":
    main()
