#!/usr/bin/env python3
"""Host-to-HBM copy rate by transfer size (the validator file path's H2D unit):
hipMemcpyAsync (torch copy_ from pinned memory, non_blocking) of a 1 GiB pinned buffer in
pieces of 1-256 MiB back to back on one stream, and alternating over two streams; best of 3."""
import json
import time

import torch


def rate(src, dst, piece, streams):
    n = src.numel()
    ss = [torch.cuda.Stream() for _ in range(streams)]
    best = 1e9
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k, o in enumerate(range(0, n, piece)):
            with torch.cuda.stream(ss[k % streams]):
                dst[o:o + piece].copy_(src[o:o + piece], non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return n / best / 1e9


def main():
    n = 1 << 30
    src = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    src.fill_(7)
    dst = torch.empty(n, dtype=torch.uint8, device="cuda")
    rate(src, dst, 64 << 20, 1)  # warm
    for mb in (1, 2, 4, 8, 16, 32, 64, 128, 256):
        print(json.dumps({"piece_mib": mb, "one_stream_gb_per_s": round(rate(src, dst, mb << 20, 1), 2),
                          "two_streams_gb_per_s": round(rate(src, dst, mb << 20, 2), 2)}), flush=True)


if __name__ == "__main__":
    main()
