"""Development probe: host->device copy bandwidth from pinned memory (the end-to-end leg's H2D),
one stream vs two, whole columns vs 8 MB pieces, and device->host beside it."""
import time

import torch


def bw(fn, nbytes, reps=5):
    torch.cuda.synchronize()
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t) / 1e9


def main():
    n = 100 << 20
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    h2 = torch.empty(16 << 20, dtype=torch.uint8, pin_memory=True)
    d2 = torch.empty(16 << 20, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    print("h2d one copy GB/s", round(bw(lambda: d.copy_(h, non_blocking=True), n), 1))

    def pieces():
        for o in range(0, n, 8 << 20):
            d[o:o + (8 << 20)].copy_(h[o:o + (8 << 20)], non_blocking=True)
    print("h2d 8 MB pieces GB/s", round(bw(pieces, n), 1))

    def two():
        with torch.cuda.stream(s1):
            d[: n // 2].copy_(h[: n // 2], non_blocking=True)
        with torch.cuda.stream(s2):
            d[n // 2:].copy_(h[n // 2:], non_blocking=True)
    print("h2d two streams GB/s", round(bw(two, n), 1))

    def duplex():
        with torch.cuda.stream(s1):
            d.copy_(h, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
    print("h2d 100 MB + d2h 16 MB duplex GB/s (h2d bytes)", round(bw(duplex, n), 1))
    print("d2h one copy GB/s", round(bw(lambda: h.copy_(d, non_blocking=True), n), 1))


if __name__ == "__main__":
    main()
