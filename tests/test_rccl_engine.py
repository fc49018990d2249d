"""The native RCCL collective engine (csrc/kernels/collective.hip, parallel/rccl.py) on one GPU.

A one-GPU box can only host one-rank RCCL communicators (RCCL refuses two ranks on one device:
"Duplicate GPU detected"), and on one rank every algorithm's plan is a single all-reduce. So
these tests check what one rank can: the engine's stream ordering (bucket launches fork from the
producing stream, `join` makes the consumer wait), the bf16 compression casts, the one-rank
identity of each algorithm's entry point, hipGraph capture of bucket launches, the bus-bandwidth
probe, BucketedAllReducer driving the engine, the watchdog turning a stalled communicator stream
into an error, and the persistent-grid CU reservation. What they do NOT run: the multi-rank
branches (reduce-scatter / all-gather / reduce / broadcast). Their per-rank call plans are
replayed against RCCL semantics on the CPU for 2..8 ranks (tests/test_collective_plan.py); the
mean-over-replicas property is covered on gloo (test_collective_multirank.py) and by the
driver's multi-GPU bench (`replicas_in_sync`).
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


def test_watchdog_aborts_a_stalled_communicator():
    """A peer that never arrives leaves the communicator stream stuck: the watchdog thread sees
    the join marker older than the deadline, aborts the communicator, and the next bucket / join
    raises (UnavailableError: what the recoverable session acts on) instead of hanging."""
    import time
    from tensorflow_train_distributed_amd.parallel import rccl
    from tensorflow_train_distributed_amd.utils import errors
    dev = torch.device("cuda", 0)
    c = rccl.RcclCommunicator(rccl.unique_id(), 1, 0, dev, timeout=1.0)
    flag = torch.zeros(1, dtype=torch.int32).pin_memory()
    try:
        # stall the communicator stream (kernel exits by itself after 20 s at the latest)
        c.debug_stall(flag.data_ptr(), 20000)
        c.join()  # arms the watchdog: the marker sits behind the stall
        t0 = time.time()
        while not c.aborted and time.time() - t0 < 10:
            time.sleep(0.05)
        assert c.aborted, "watchdog did not abort within 10 s"
        assert 0.8 < time.time() - t0 < 10
        x = torch.zeros(1024, device=dev)
        with pytest.raises(errors.UnavailableError):
            c.bucket(x)
        with pytest.raises(errors.UnavailableError):
            c.join()
        assert "no progress" in c.error
    finally:
        flag[0] = 1  # release the stall kernel
        torch.cuda.synchronize()
        c.destroy(abort=True)


def test_persistent_grids_follow_the_cu_reservation():
    from tensorflow_train_distributed_amd.parallel import rccl
    total = torch.cuda.get_device_properties(0).multi_processor_count
    old = rccl.set_reserved_cus(8)
    try:
        assert rccl.persistent_cus() == total - 8
        # the persistent kernels still compute the same thing on fewer CUs
        from tensorflow_train_distributed_amd.ops import gemm as G
        a = torch.randn(65536, 1024, device="cuda").bfloat16()  # 1024 tiles: the persistent kernel
        b = torch.randn(1024, 1024, device="cuda").bfloat16()
        ref = (a.float() @ b.float())
        out = G.gemm(a, b)
        rel = float((out.float() - ref).norm() / ref.norm())
        assert rel < 1e-2, rel
    finally:
        rccl.set_reserved_cus(old)
    assert rccl.persistent_cus() == total


def test_segmented_capture_with_bucket_launches_matches_eager():
    """N>1's hipGraph: under utils.graphs.capture_segmented the reducer's bucket forks and its
    final join become event nodes and the communicator stream records its own linear graph
    segments (parallel/collective.py). On a one-rank native communicator the replayed step
    (gradients produced on a side stream, buckets launched as they become final, the optimizer-
    like consumer on the main stream after finish()) matches the eager step bitwise, the
    bucket launches are in the graph (a replay re-reduces fresh data), and arming the watchdog
    after a replay leaves the engine healthy."""
    import torch.distributed as dist
    from tensorflow_train_distributed_amd.parallel.collective import BucketedAllReducer
    from tensorflow_train_distributed_amd.train.flat import FlatParams, ParamSpec
    from tensorflow_train_distributed_amd.utils import graphs
    assert not dist.is_initialized()
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    try:
        sizes = [20000, 3, 1200000, 5000, 250000]
        specs = [ParamSpec("v%d" % i, (n,), None, True) for i, n in enumerate(sizes)]
        p = FlatParams(specs, dev, compute_dtype=None)
        red = BucketedAllReducer(p, bucket_mb=1.0, first_bucket_mb=0.05, compress_bf16=True, engine="native")
        assert red.engine == "native-rccl" and len(red.buckets) >= 3
        src = torch.randn(p.numel, device=dev) * p.valid_mask().to(dev)
        out = torch.zeros(p.numel, device=dev)
        side = torch.cuda.Stream(device=dev)
        main = torch.cuda.Stream(device=dev)

        def step():
            red.begin()
            cur = torch.cuda.current_stream()
            graphs.fork(cur, side)
            with torch.cuda.stream(side):
                for s in specs:  # "backward": each gradient final, then its buckets launch
                    o, n = p.offsets[s.name], s.shape[0]
                    p.grad[o:o + n].copy_(src[o:o + n] * 2.0)
                    red.mark_ready(s.name)
            graphs.join(cur, side)
            red.finish()
            out.copy_(p.grad * 3.0)  # consumer after the collectives
            return out

        with torch.cuda.stream(main):
            step()
        torch.cuda.synchronize()
        eager = out.clone()
        torch.testing.assert_close(eager, (src * 2.0).bfloat16().float() * 3.0, rtol=0, atol=0)
        seg = graphs.capture_segmented(step, main=main, warmup=1)
        assert seg.info["streams"] >= 3, seg.info  # main, side and the communicator stream
        out.zero_()
        p.grad.zero_()
        seg.replay()
        red.comm.arm(main)
        torch.cuda.synchronize()
        assert torch.equal(out, eager)
        src.mul_(-0.5)  # fresh data: the replayed buckets must reduce (cast) it again
        seg.replay()
        red.comm.arm(main)
        torch.cuda.synchronize()
        torch.testing.assert_close(out, (src * 2.0).bfloat16().float() * 3.0, rtol=0, atol=0)
        assert not red.comm.aborted
    finally:
        from tensorflow_train_distributed_amd.parallel import rccl
        rccl.abort_all()
        dist.destroy_process_group()


def test_cta_budget_probe_path_on_one_rank(monkeypatch):
    """The start-up CTA-budget probe (rccl._probe_budgets) end to end on a one-rank RCCL group
    (TTD_RCCL_PROBE=force): two communicators (capped / RCCL default) created and probed, the
    slowest-rank table agreed over the process group, the policy's choice kept (the other
    communicator finalized), the reducer reporting it."""
    import torch.distributed as dist
    from tensorflow_train_distributed_amd.parallel import rccl
    from tensorflow_train_distributed_amd.parallel.collective import BucketedAllReducer
    from tensorflow_train_distributed_amd.train.flat import FlatParams, ParamSpec
    monkeypatch.setenv("TTD_RCCL_PROBE", "force")
    monkeypatch.delenv("TTD_RCCL_MAX_CTAS", raising=False)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    try:
        specs = [ParamSpec("v%d" % i, (n,), None, True) for i, n in enumerate([300000, 5000, 900000])]
        p = FlatParams(specs, dev, compute_dtype=None)
        red = BucketedAllReducer(p, bucket_mb=1.0, first_bucket_mb=0.5, engine="native", overlap_ms=40.0)
        pol = red.policy()
        assert pol is not None and pol["cta_budget"] in (0, rccl.DEFAULT_MAX_CTAS), pol
        assert set(pol["probe"]) == {rccl.DEFAULT_MAX_CTAS, 0}
        for rows in pol["probe"].values():
            assert [r["bytes"] for r in rows] == list(rccl.PROBE_BYTES) and all(r["ms"] > 0 for r in rows)
        assert red.comm.max_ctas == pol["cta_budget"]
        # the kept communicator works
        local = torch.randn(p.numel, device=dev) * p.valid_mask().to(dev)
        p.grad.copy_(local)
        red.begin()
        for s in specs:
            red.mark_ready(s.name)
        red.finish()
        torch.cuda.synchronize()
        torch.testing.assert_close(p.grad, local, rtol=0, atol=0)
    finally:
        rccl.abort_all()
        dist.destroy_process_group()
