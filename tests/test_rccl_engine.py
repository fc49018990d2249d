"""The native RCCL collective engine (csrc/kernels/collective.hip, parallel/rccl.py) on one GPU.

A one-GPU box can only host one-rank RCCL communicators (RCCL refuses two ranks on one device:
"Duplicate GPU detected"), so these tests check what one rank can: the engine's stream ordering
(bucket launches fork from the producing stream, `join` makes the consumer wait), the bf16
compression casts, every reduction algorithm's code path, hipGraph capture of bucket
launches, the bus-bandwidth probe, and BucketedAllReducer driving the engine. The N-rank
arithmetic (mean over replicas, bucket order) is covered on gloo by test_collective_multirank.py
over the same BucketedAllReducer, and by the driver's multi-GPU bench (`replicas_in_sync`).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    from tensorflow_train_distributed_amd.parallel import rccl
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c = rccl.RcclCommunicator(rccl.unique_id(), 1, 0, dev)
    yield c
    c.destroy()


def _slow_then(fn):
    """Queue a long GEMM chain on the current stream, then fn(): a consumer that does not wait
    for the current stream would read fn's inputs before they are written."""
    a = torch.randn(4096, 4096, device="cuda")
    for _ in range(8):
        a = a @ a
        a = a / a.norm()
    return fn()


def test_version_and_single_rank_identity(comm):
    from tensorflow_train_distributed_amd.parallel import rccl
    assert rccl.rccl_version() >= 22000
    x = torch.randn(1 << 20, device="cuda")
    ref = x.clone()
    for algo in ("allreduce", "hierarchical", "reduce_to_one"):
        for op in ("sum", "avg"):
            comm.bucket(x, op=op, algorithm=algo)
    comm.join()
    torch.testing.assert_close(x, ref, rtol=0, atol=0)
    i = torch.arange(1000, dtype=torch.int64, device="cuda")
    comm.all_reduce_(i, op="max")
    d = torch.randn(333, dtype=torch.float64, device="cuda")
    dref = d.clone()
    comm.broadcast_(d, root=0)
    torch.cuda.synchronize()
    assert torch.equal(i, torch.arange(1000, dtype=torch.int64, device="cuda")) and torch.equal(d, dref)


def test_bucket_orders_after_producer_and_join_orders_consumer(comm):
    n = (1 << 22) + 5  # odd tail for the vectorised casts
    y = torch.randn(n, device="cuda")
    x = torch.zeros(n, device="cuda")
    # producer: x <- y behind a long chain; the compressed bucket casts x on the communicator
    # stream, so it must see y (ordering), and the consumer after join must see the round trip
    _slow_then(lambda: x.copy_(y))
    comm.bucket(x, compress=True)
    comm.join()
    z = x * 2
    torch.cuda.synchronize()
    want = y.bfloat16().float()
    assert torch.equal(x, want)
    assert torch.equal(z, want * 2)


def test_bucket_launches_capture_in_a_hipgraph(comm):
    n = 3 << 18
    y = torch.randn(n, device="cuda")
    x = torch.zeros(n, device="cuda")
    out = torch.zeros(n, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())

    def body():
        x.copy_(y)
        comm.bucket(x[: n // 2], compress=True)
        comm.bucket(x[n // 2:], algorithm="hierarchical")
        comm.join()
        out.copy_(x * 3)

    with torch.cuda.stream(s):  # warm-up (sizes the bf16 staging buffer outside capture)
        body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        body()
    for _ in range(2):
        y.copy_(torch.randn(n, device="cuda"))
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        want = torch.cat([y[: n // 2].bfloat16().float(), y[n // 2:]]) * 3
        assert torch.equal(out, want)


def test_probe_reports_time(comm):
    r = comm.probe(8 << 20, iters=3)
    assert r["bytes"] == 8 << 20 and r["ms"] > 0


def test_bucketed_allreducer_drives_the_engine():
    """BucketedAllReducer(engine="native") on a one-rank RCCL process group: buckets launch as
    their variables become final, go through the native communicator, and finish() orders the
    optimizer's stream after them."""
    import torch.distributed as dist
    from tensorflow_train_distributed_amd.parallel.collective import BucketedAllReducer
    from tensorflow_train_distributed_amd.train.flat import FlatParams, ParamSpec
    assert not dist.is_initialized()
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    try:
        specs = [ParamSpec("v%d" % i, (n,), None, True) for i, n in enumerate([20000, 3, 1200000, 5000, 250000])]
        p = FlatParams(specs, dev, compute_dtype=None)
        red = BucketedAllReducer(p, bucket_mb=1.0, first_bucket_mb=0.05, compress_bf16=True, engine="native")
        assert red.engine == "native-rccl" and len(red.buckets) >= 3
        local = torch.randn(p.numel, device=dev) * p.valid_mask().to(dev)
        red.begin()
        for s in specs:
            o, n = p.offsets[s.name], s.shape[0]
            _slow_then(lambda: p.grad[o:o + n].copy_(local[o:o + n]))
            red.mark_ready(s.name)
        red.finish()
        after = p.grad * 1.0  # consumer on the current stream
        torch.cuda.synchronize()
        assert red.launch_log == list(range(len(red.buckets)))
        torch.testing.assert_close(after, local.bfloat16().float(), rtol=0, atol=0)
        # instrumented step: per-bucket busy time on the communicator stream + exposed time
        assert red.time_next_step()
        red.begin()
        for s in specs:
            red.mark_ready(s.name)
        red.finish()
        st = red.comm_stats()
        assert st["buckets"] == len(red.buckets) and st["busy_ms"] > 0 and st["span_ms"] >= 0
        assert st["exposed_ms"] >= 0 and 0 <= st["overlap_pct"] <= 100
    finally:
        from tensorflow_train_distributed_amd.parallel import rccl
        rccl.abort_all()
        dist.destroy_process_group()
