#!/usr/bin/env python3
"""Does a hipGraph replay keep two captured streams concurrent? Two independent chains of
kernels (one per stream, forked from and joined to the capture stream); compares the eager
two-stream time, the eager serial time and the graph replay time."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402


def main():
    dev = "cuda"
    # small GEMMs that each fill only part of the chip (the side-stream wgrad situation)
    a = torch.randn(2048, 1024, device=dev).bfloat16()
    b = torch.randn(1024, 256, device=dev).bfloat16()
    c = torch.randn(2048, 1024, device=dev).bfloat16()
    d = torch.randn(1024, 256, device=dev).bfloat16()
    side = torch.cuda.Stream()
    n = 40

    def work(concurrent):
        main = torch.cuda.current_stream()
        if concurrent:
            ev = torch.cuda.Event()
            ev.record()
            side.wait_event(ev)
            with torch.cuda.stream(side):
                for _ in range(n):
                    G.gemm(c, d)
        for _ in range(n):
            G.gemm(a, b)
        if concurrent:
            main.wait_stream(side)
        else:
            for _ in range(n):
                G.gemm(c, d)

    def timeit(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps

    t_ser = timeit(lambda: work(False))
    t_con = timeit(lambda: work(True))
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        work(True)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            work(True)
    torch.cuda.synchronize()
    t_graph = timeit(g.replay)
    print("eager serial %.3f ms  eager 2-stream %.3f ms  graph replay %.3f ms" % (t_ser, t_con, t_graph), flush=True)


if __name__ == "__main__":
    main()
