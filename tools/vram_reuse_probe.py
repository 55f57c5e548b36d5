#!/usr/bin/env python3
"""Cold-memory probe: what does the first touch of device memory cost when it
is freshly allocated vs when it reuses VRAM another allocation just freed?
(bench.py's general path once paid 858 ms in its first join after the
headline's buffers were freed.)  Caching allocator off: every free is a
hipFree, every empty a hipMalloc.  One JSON line per step."""
import json
import os
import time

os.environ["PYTORCH_NO_CUDA_MEMORY_CACHING"] = "1"
import torch  # noqa: E402


def step(name, fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    print(json.dumps({"step": name, "ms": round((time.perf_counter() - t0) * 1e3, 3)}), flush=True)
    return r


def main():
    gb = float(os.environ.get("PROBE_GB", "40"))
    n = int(gb * 1e9)
    a = step("alloc_fresh", lambda: torch.empty(n, dtype=torch.uint8, device="cuda"))
    step("fill_fresh", lambda: a.fill_(1))
    step("fill_warm", lambda: a.fill_(2))
    del a
    step("free", lambda: None)
    b = step("alloc_reuse", lambda: torch.empty(n, dtype=torch.uint8, device="cuda"))
    step("fill_reuse", lambda: b.fill_(1))
    step("fill_reuse_warm", lambda: b.fill_(2))
    c = step("alloc_fresh2", lambda: torch.empty(n, dtype=torch.uint8, device="cuda"))
    step("fill_fresh2", lambda: c.fill_(1))
    del b, c
    time.sleep(2.0)
    d = step("alloc_after_sleep", lambda: torch.empty(n, dtype=torch.uint8, device="cuda"))
    step("fill_after_sleep", lambda: d.fill_(1))


if __name__ == "__main__":
    main()
