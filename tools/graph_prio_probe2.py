#!/usr/bin/env python3
"""Does a hipGraph replayed on a high-priority stream keep that stream's priority?

A normal-priority "side" stream is loaded with long, chip-filling elementwise kernels; a
high-priority "main" stream then runs a chain of small kernels. With priority honoured, the
main chain's workgroups dispatch ahead of the side stream's queued ones and the chain ends
early. The chain's completion time (from its first launch) is measured eagerly and with each
stream's work replayed as its own captured graph on the same streams (what
utils.graphs.capture_segmented does), plus both at equal (normal) priority for reference.

    python tools/graph_prio_probe2.py
"""
import json
import time

import torch


def main():
    dev = torch.device("cuda", 0)
    lo, hi = torch.cuda.Stream.priority_range()
    big = torch.empty(1 << 28, device=dev)  # 1 GB
    small = torch.zeros(1 << 16, device=dev)

    def side_work():
        for _ in range(12):
            big.mul_(1.0000001)

    def main_work():
        for _ in range(300):
            small.add_(1.0)

    res = {}
    for prio_name, mprio in (("high", hi), ("equal", lo)):
        side = torch.cuda.Stream(device=dev, priority=lo)
        mainst = torch.cuda.Stream(device=dev, priority=mprio)
        # graphs
        gs, gm = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        for s, g, fn in ((side, gs, side_work), (mainst, gm, main_work)):
            with torch.cuda.stream(s):
                fn()  # warm-up
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                fn()
        torch.cuda.synchronize()
        for mode in ("eager", "graph"):
            ts = []
            for rep in range(6):
                e0 = torch.cuda.Event(enable_timing=True)
                e_side = torch.cuda.Event(enable_timing=True)
                e_main = torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record(side)
                if mode == "eager":
                    with torch.cuda.stream(side):
                        side_work()
                    mainst.wait_event(e0)
                    with torch.cuda.stream(mainst):
                        main_work()
                else:
                    with torch.cuda.stream(side):
                        gs.replay()
                    mainst.wait_event(e0)
                    with torch.cuda.stream(mainst):
                        gm.replay()
                e_side.record(side)
                e_main.record(mainst)
                torch.cuda.synchronize()
                if rep >= 2:
                    ts.append((e0.elapsed_time(e_main), e0.elapsed_time(e_side)))
            res["%s/%s" % (prio_name, mode)] = {"main_done_ms": round(min(t[0] for t in ts), 3),
                                                "side_done_ms": round(min(t[1] for t in ts), 3)}
            print(prio_name, mode, res["%s/%s" % (prio_name, mode)], flush=True)
    # main chain alone
    mainst = torch.cuda.Stream(device=dev, priority=hi)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(mainst)
    with torch.cuda.stream(mainst):
        main_work()
    e1.record(mainst)
    torch.cuda.synchronize()
    res["main_alone_ms"] = round(e0.elapsed_time(e1), 3)
    print(json.dumps(res))


if __name__ == "__main__":
    t = time.time()
    main()
