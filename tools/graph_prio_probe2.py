#!/usr/bin/env python3
"""Probe 2: can a replayed hipGraph keep a two-stream step's main-chain priority?

Round 2's probe (graph_prio_probe.py) set the priority attribute on the first node of the
graph without checking that it was a kernel node. Here:
  1. capture a two-stream workload (main: a latency-bound chain of small GEMMs; side: large
     bandwidth-bound kernels) with torch.cuda.CUDAGraph(keep_graph=True), tagging the side
     stream's nodes during capture (graphs.side_scope: node-set difference around the block);
  2. set hipLaunchAttributePriority on every KERNEL node (main high, side low) and instantiate
     with hipGraphInstantiateFlagUseNodePriority;
  3. time: eager (main on a high-priority stream), plain replay, node-priority replay.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tensorflow_train_distributed_amd.utils import graphs  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    lo, hi = torch.cuda.Stream.priority_range()
    main_s = torch.cuda.Stream(priority=hi)
    side = torch.cuda.Stream(priority=lo)
    a = torch.randn(2048, 2048, device=dev).bfloat16()
    w = torch.randn(2048, 2048, device=dev).bfloat16() / 45
    big = torch.randn(1 << 28, device=dev).bfloat16()
    out_big = torch.empty_like(big)

    def step():
        x = a
        ev = torch.cuda.Event()
        ev.record()
        side.wait_event(ev)
        with graphs.side_scope(side):
            with torch.cuda.stream(side):
                for _ in range(6):
                    torch.mul(big, 1.0001, out=out_big)
                    torch.add(out_big, 1.0, out=big)
        for _ in range(120):
            x = torch.relu(x @ w)
        torch.cuda.current_stream().wait_stream(side)
        return x

    def timeit(fn, n=10):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    res = {}
    main_s.wait_stream(torch.cuda.current_stream())

    def eager():
        with torch.cuda.stream(main_s):
            step()
    res["eager_two_prio_ms"] = timeit(eager)

    def main_only():
        with torch.cuda.stream(main_s):
            x = a
            for _ in range(120):
                x = torch.relu(x @ w)
    res["main_chain_alone_ms"] = timeit(main_only)

    g = graphs.capture_prioritized(step, stream=main_s)
    res["nodes"] = g.info
    res["graph_plain_ms"] = timeit(g.replay_plain)
    if g.prio_exec is not None:
        res["graph_node_prio_ms"] = timeit(g.replay)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
