"""Diagnostic: the cost of HIP events' system-scope fences between HBM-heavy kernels.

Each iteration writes a 2 GiB buffer (one fill kernel on stream A) and, per variant:
  plain     nothing else
  sync      record a sync event on A and make A wait on an event recorded on stream B
            (the pipeline's pattern), torch events (hipEventDisableTiming: system fence)
  sync_nf   the same with hipEventDisableTiming | hipEventDisableSystemFence events
  timing    two timing events around the kernel (hipEventCreate: system fence; the
            library's tmh_profile events)
  timing_nf the same with hipEventDisableSystemFence
A second stream B runs small L2-resident kernels beside it (a 4 MiB buffer re-read), whose
throughput shows what the fences' L2 writeback / invalidation costs a neighbour.
Usage (GPU box): python scripts/micro/event_fence.py
"""
import ctypes as C
import time

import torch

hip = C.CDLL("libamdhip64.so.7")
hip.hipEventCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
hip.hipStreamWaitEvent.argtypes = [C.c_void_p, C.c_void_p, C.c_uint]
DISABLE_TIMING, NO_FENCE = 0x2, 0x20000000


def ev(flags):
    e = C.c_void_p()
    assert hip.hipEventCreateWithFlags(C.byref(e), flags) == 0
    return e


def main():
    dev = torch.device("cuda:0")
    big = torch.empty(2 << 30, dtype=torch.uint8, device=dev)
    small = torch.ones(1 << 20, dtype=torch.float32, device=dev)
    acc = torch.zeros(1, dtype=torch.float32, device=dev)
    A, B = torch.cuda.Stream(), torch.cuda.Stream()
    ha, hb = C.c_void_p(A.cuda_stream), C.c_void_p(B.cuda_stream)
    n = 60

    def run(variant):
        evs = {"sync": (ev(DISABLE_TIMING), ev(DISABLE_TIMING)), "sync_nf": (ev(DISABLE_TIMING | NO_FENCE), ev(DISABLE_TIMING | NO_FENCE)),
               "timing": (ev(0), ev(0)), "timing_nf": (ev(NO_FENCE), ev(NO_FENCE))}.get(variant)
        torch.cuda.synchronize()
        nb = 0
        t0 = time.perf_counter()
        for i in range(n):
            with torch.cuda.stream(A):
                if variant.startswith("timing"):
                    hip.hipEventRecord(evs[0], ha)
                big.fill_(i & 255)
                if variant.startswith("timing"):
                    hip.hipEventRecord(evs[1], ha)
                if variant.startswith("sync"):
                    hip.hipEventRecord(evs[0], ha)
                    hip.hipEventRecord(evs[1], hb)
                    hip.hipStreamWaitEvent(ha, evs[1], 0)
            with torch.cuda.stream(B):
                for _ in range(4):
                    acc.add_(small.sum())
                    nb += 1
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        return dt / n * 1e6, nb / dt

    for v in ("plain", "sync", "sync_nf", "timing", "timing_nf"):
        run(v)   # warm
    for rep in range(2):
        for v in ("plain", "sync", "sync_nf", "timing", "timing_nf"):
            us, rb = run(v)
            print(f"{v:10s} {us:8.1f} us per 2 GiB fill   neighbour {rb:9.0f} small kernels/s")


if __name__ == "__main__":
    main()
