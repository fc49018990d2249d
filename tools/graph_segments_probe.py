#!/usr/bin/env python3
"""Probe: a two-stream step captured as two concurrently recorded LINEAR hipGraphs (one per
stream) whose cross-stream dependencies are external event record / wait nodes
(hipEventRecordExternal / hipEventWaitExternal), replayed on the original main (high priority)
and side (normal priority) streams.

Checks (1) replay computes what eager computes, (2) replay time vs eager. The workload: a main
chain of small GEMMs forks a side branch (bandwidth-heavy elementwise work) twice and joins it.
To keep every wait enqueued after its record, the capture is cut at each join into segments
launched in capture order (main_k, side_k, main_k+1, ...)."""
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
P = ctypes.c_void_p


def ev_new():
    e = P(0)
    assert hip.hipEventCreateWithFlags(ctypes.byref(e), 2) == 0  # hipEventDisableTiming
    return e


def _capture_state(stream):
    status, cid, graph, deps, n = ctypes.c_int(0), ctypes.c_ulonglong(0), P(0), P(0), ctypes.c_size_t(0)
    rc = hip.hipStreamGetCaptureInfo_v2(P(stream.cuda_stream), ctypes.byref(status), ctypes.byref(cid),
                                        ctypes.byref(graph), ctypes.byref(deps), ctypes.byref(n))
    assert rc == 0 and status.value == 1, (rc, status.value)
    return graph, deps, n


def _add_node(stream, ev, adder):
    # hipEventRecordWithFlags(..., hipEventRecordExternal) is refused under capture on ROCm 7.2
    # (hipErrorInvalidValue): add the event node to the capture graph by hand, after the stream's
    # current dependencies, and make it the stream's new dependency set
    graph, deps, n = _capture_state(stream)
    node = P(0)
    rc = adder(ctypes.byref(node), graph, deps, n, ev)
    assert rc == 0, rc
    rc = hip.hipStreamUpdateCaptureDependencies(P(stream.cuda_stream), ctypes.byref(node), ctypes.c_size_t(1), 1)
    assert rc == 0, rc


def rec_ext(ev, stream):
    _add_node(stream, ev, hip.hipGraphAddEventRecordNode)


def wait_ext(stream, ev):
    _add_node(stream, ev, hip.hipGraphAddEventWaitNode)


def main():
    dev = torch.device("cuda", 0)
    lo, hi = torch.cuda.Stream.priority_range()
    main_s = torch.cuda.Stream(priority=hi)
    side = torch.cuda.Stream(priority=lo)
    a = torch.randn(2048, 2048, device=dev).bfloat16()
    w = torch.randn(2048, 2048, device=dev).bfloat16() / 45
    big = torch.randn(1 << 27, device=dev)
    out_big = torch.empty_like(big)
    res = torch.zeros(2048, 2048, device=dev)
    evs = [ev_new() for _ in range(8)]

    def body(mode, seg=None):
        """mode 'eager' (torch events) or 'graph' (external events, seg(k) cuts segments)."""
        x = a
        for part in range(2):
            if mode == "eager":
                e = torch.cuda.Event()
                e.record()
                side.wait_event(e)
            else:
                rec_ext(evs[2 * part], main_s)
                wait_ext(side, evs[2 * part])
            with torch.cuda.stream(side):
                for _ in range(3):
                    torch.mul(big, 1.0001, out=out_big)
                    torch.add(out_big, 1.0, out=big)
                res.add_(big[: 2048 * 2048].view(2048, 2048))
            for _ in range(60):
                x = torch.relu(x @ w)
            if mode == "eager":
                torch.cuda.current_stream().wait_stream(side)
            else:
                rec_ext(evs[2 * part + 1], side)
                seg()  # cut: the join's wait starts the next main segment
                wait_ext(main_s, evs[2 * part + 1])
        res.add_(x.float())

    def run_eager():
        with torch.cuda.stream(main_s):
            body("eager")

    # eager reference
    big_init = big.clone()
    res.zero_()
    run_eager()
    torch.cuda.synchronize()
    want = res.clone()

    # segmented capture: main and side each record one linear graph per segment
    # one private memory pool per stream (torch refuses two concurrent captures into one pool);
    # sequential segments of a stream share its pool and replay in capture order
    pools = {main_s: torch.cuda.graph_pool_handle(), side: torch.cuda.graph_pool_handle()}
    graphs = []  # (stream, graph) in capture order
    cur = {}

    def begin():
        for s in (main_s, side):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                g.capture_begin(pool=pools[s], capture_error_mode="relaxed")
            cur[s] = g

    def end():
        for s in (main_s, side):  # main segment first (its forks precede the side's waits)
            with torch.cuda.stream(s):
                cur[s].capture_end()
            graphs.append((s, cur[s]))

    def seg():
        end()
        begin()

    main_s.wait_stream(torch.cuda.current_stream())
    side.wait_stream(torch.cuda.current_stream())
    torch.cuda.synchronize()
    big.copy_(big_init)
    res.zero_()
    begin()
    with torch.cuda.stream(main_s):
        body("graph", seg)
    end()
    torch.cuda.synchronize()

    def replay():
        for s, g in graphs:
            with torch.cuda.stream(s):
                g.replay()

    big.copy_(big_init)
    res.zero_()
    torch.cuda.synchronize()
    replay()
    torch.cuda.synchronize()
    ok = bool(torch.allclose(res, want, rtol=1e-3, atol=1e-3))

    def timeit(fn, n=10):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    out = {"segments": len(graphs), "replay_matches_eager": ok, "eager_ms": round(timeit(run_eager), 3),
           "segmented_graph_ms": round(timeit(replay), 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
