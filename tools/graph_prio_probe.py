"""Probe: does hipStreamBeginCapture record the capturing stream's priority on kernel nodes,
and does a graph instantiated with hipGraphInstantiateFlagUseNodePriority honour them?

  python tools/graph_prio_probe.py           # tiny two-stream capture, prints node priorities

Result on MI355X / ROCm 7 (this image): every captured kernel node reads priority 0 (the
high-priority capturing stream's -1 is not recorded), and hipGraphKernelNodeSetAttribute with
hipLaunchAttributePriority returns hipErrorInvalidValue, so a replay cannot keep the eager
step's main-chain-over-weight-gradient priority (ResNet-50 b1024 on one box: eager 74.9 ms,
graph replay 78.6 ms). The bench therefore stays eager.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
P = ctypes.c_void_p


def nodes(graph):
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(P(graph), None, ctypes.byref(n)) == 0
    arr = (P * n.value)()
    assert hip.hipGraphGetNodes(P(graph), arr, ctypes.byref(n)) == 0
    return list(arr)


def prio_hist(graph):
    hist = {}
    for nd in nodes(graph):
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(P(nd), ctypes.byref(t))
        if t.value != 0:  # kernel nodes only
            continue
        v = (ctypes.c_char * 128)()
        rc = hip.hipGraphKernelNodeGetAttribute(P(nd), 8, v)  # hipLaunchAttributePriority
        pr = ctypes.cast(v, ctypes.POINTER(ctypes.c_int))[0] if rc == 0 else ("rc%d" % rc)
        hist[pr] = hist.get(pr, 0) + 1
    return hist


def main():
    lo, hi = torch.cuda.Stream.priority_range()
    print("priority range", lo, hi)
    main_s = torch.cuda.Stream(priority=hi)
    side = torch.cuda.Stream()
    x = torch.randn(1024, 1024, device="cuda")
    y = torch.randn(1024, 1024, device="cuda")
    g = torch.cuda.CUDAGraph(keep_graph=True)
    main_s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=main_s):
        a = x * 2
        ev = torch.cuda.Event()
        ev.record()
        side.wait_event(ev)
        with torch.cuda.stream(side):
            b = y * 3
            b = b + 1
        a = a + 1
        torch.cuda.current_stream().wait_stream(side)
        c = a + b
    print("kernel-node priorities:", prio_hist(g.raw_cuda_graph()))
    # setting a node priority by hand (what a priority-aware replay would need)
    nd = [n for n in nodes(g.raw_cuda_graph())][0]
    v = (ctypes.c_char * 128)()
    ctypes.cast(v, ctypes.POINTER(ctypes.c_int))[0] = hi
    print("hipGraphKernelNodeSetAttribute(priority) rc =", hip.hipGraphKernelNodeSetAttribute(P(nd), 8, v))


if __name__ == "__main__":
    main()
