"""N-rank arithmetic of the native collective engine, on the CPU.

A one-GPU box can only host one-rank RCCL communicators, where the engine's plan is a single
all-reduce. The per-rank call sequences of the multi-rank algorithms (hierarchical reduce-scatter
+ all-gather with the count % nranks tail, reduce-to-one + broadcast) come from one host function
(csrc/kernels/collective_plan.h) that collective.hip executes verbatim and libttd_rt.so exports.
Here every rank's plan is replayed with RCCL's semantics on numpy buffers, for 2..8 ranks and
ragged counts: the plans must match call-for-call across ranks (otherwise RCCL would pair
different collectives) and leave the elementwise sum on every rank.

Also: the co-scheduling hooks of BucketedAllReducer (persistent grids leave the CTA budget's CUs
to the collectives from the first bucket launch to finish()).
"""
import ctypes

import numpy as np
import pytest

ALLREDUCE, REDUCE_SCATTER, ALL_GATHER, REDUCE, BROADCAST = range(5)


def _plan(algo, count, nranks, rank):
    from tensorflow_train_distributed_amd import _native
    lib = _native.rt()
    n_max = lib.ttd_collective_plan_max_steps()
    out = (ctypes.c_longlong * (5 * n_max))()
    n = lib.ttd_collective_plan(int(algo), ctypes.c_longlong(count), int(nranks), int(rank), out)
    assert n >= 0
    return [tuple(out[5 * i:5 * i + 5]) for i in range(n)]


def _simulate(algo, count, nranks, seed=0):
    rng = np.random.default_rng(seed)
    bufs = [rng.integers(-1000, 1000, size=count).astype(np.int64) for _ in range(nranks)]
    want = sum(bufs)
    plans = [_plan(algo, count, nranks, r) for r in range(nranks)]
    # the same sequence of collectives (kind, root, count) on every rank
    shape = [[(k, root, c) for k, root, _, _, c in p] for p in plans]
    assert all(s == shape[0] for s in shape), shape
    for step in range(len(plans[0])):
        kind, root, _, _, c = plans[0][step]
        send = [plans[r][step][2] for r in range(nranks)]
        recv = [plans[r][step][3] for r in range(nranks)]
        if kind == ALLREDUCE:
            assert len(set(send)) == 1  # in place on the same slice everywhere
            s = sum(b[send[0]:send[0] + c] for b in bufs)
            for b in bufs:
                b[send[0]:send[0] + c] = s
        elif kind == REDUCE_SCATTER:
            full = sum(b[send[r]:send[r] + c * nranks] for r, b in enumerate(bufs))
            for r, b in enumerate(bufs):
                b[recv[r]:recv[r] + c] = full[r * c:(r + 1) * c]
        elif kind == ALL_GATHER:
            chunks = [b[send[r]:send[r] + c].copy() for r, b in enumerate(bufs)]
            for r, b in enumerate(bufs):
                b[recv[r]:recv[r] + c * nranks] = np.concatenate(chunks)
        elif kind == REDUCE:
            s = sum(b[send[r]:send[r] + c] for r, b in enumerate(bufs))
            bufs[root][send[root]:send[root] + c] = s
        elif kind == BROADCAST:
            src = bufs[root][send[root]:send[root] + c].copy()
            for r, b in enumerate(bufs):
                b[send[r]:send[r] + c] = src
        else:
            raise AssertionError(kind)
    return bufs, want, plans


@pytest.mark.parametrize("algo", [0, 1, 2])
@pytest.mark.parametrize("nranks", [1, 2, 3, 4, 7, 8])
@pytest.mark.parametrize("count", [1, 5, 8, 1000, 4097, 65536 + 3])
def test_every_rank_ends_with_the_sum(algo, nranks, count):
    bufs, want, plans = _simulate(algo, count, nranks, seed=count + 31 * nranks)
    for b in bufs:
        np.testing.assert_array_equal(b, want)
    if nranks == 1:
        assert [p[0] for p in plans[0]] == [ALLREDUCE]


def test_hierarchical_chunks_and_tail():
    # 8 ranks, 1003 elements: 125 per rank, the 3-element tail in one small all-reduce
    for r in range(8):
        p = _plan(1, 1003, 8, r)
        assert p == [(REDUCE_SCATTER, 0, 0, r * 125, 125), (ALL_GATHER, 0, r * 125, 0, 125),
                     (ALLREDUCE, 0, 1000, 1000, 3)]
    # fewer elements than ranks: only the all-reduce of the whole bucket
    assert _plan(1, 5, 8, 3) == [(ALLREDUCE, 0, 0, 0, 5)]
    assert _plan(1, 0, 8, 3) == []
    assert _plan(2, 10, 4, 1) == [(REDUCE, 0, 0, 0, 10), (BROADCAST, 0, 0, 0, 10)]


def test_reducer_reserves_cus_while_buckets_are_in_flight(monkeypatch):
    """From the first bucket launch to finish(), persistent kernels leave the communicator's CTA
    budget of CUs free (rccl.set_reserved_cus), and only then."""
    import torch
    from tensorflow_train_distributed_amd.parallel import collective, rccl
    from tensorflow_train_distributed_amd.train.flat import FlatParams, ParamSpec
    calls = []
    monkeypatch.setattr(rccl, "set_reserved_cus", lambda n: calls.append(n) or 0)

    class FakeComm:
        max_ctas = 8
        launched = []

        def bucket(self, t, **kw):
            self.launched.append(t.numel())

        def join(self):
            calls.append("join")

    specs = [ParamSpec("v%d" % i, (n,), None, True) for i, n in enumerate([300000, 3, 600000])]
    p = FlatParams(specs, "cpu", compute_dtype=None)
    red = collective.BucketedAllReducer(p, bucket_mb=1.0, first_bucket_mb=0.5)
    red.comm = FakeComm()
    red.reserved_cus = 8
    red.begin()
    assert calls == []  # the forward runs on every CU
    red.mark_ready("v0")
    assert calls == [8]
    red.mark_ready("v1")
    red.mark_ready("v2")
    red.finish()
    assert calls == [8, 0, "join"] and len(FakeComm.launched) == len(red.buckets)


def _probe(ms_1m, ms_32m, world):
    def row(nb, ms):
        return {"bytes": nb, "ms": ms, "busbw_GBps": round(2.0 * (world - 1) / world * nb / (ms * 1e-3) / 1e9, 1)}
    return [row(1 << 20, ms_1m), row(32 << 20, ms_32m)]


def test_cta_budget_policy_from_synthetic_probes():
    """rccl.choose_cta_budget: the capped budget stays only when the projected per-step
    all-reduce time at ITS measured bandwidth (x1.5 margin) fits the backward; otherwise RCCL's
    own budget. Without an overlap estimate the bandwidth ratio decides."""
    from tensorflow_train_distributed_amd.parallel import rccl
    w = 8
    buckets = [4 << 20] + [32 << 20] * 3 + [5 << 20]  # ResNet-50: ~105 MB of fp32 gradients
    # 8 CTAs at ~150 GB/s bus bandwidth, default at ~300 GB/s: 105 MB needs ~1.4 ms capped
    fast = {8: _probe(0.03, 0.39, w), 0: _probe(0.025, 0.195, w)}
    pol = rccl.choose_cta_budget(fast, buckets, w, overlap_ms=44.0)
    assert pol["cta_budget"] == 8 and "hides" in pol["reason"]
    assert 1.0 < pol["projected_ms"]["8"] < 2.5 and pol["projected_ms"]["0"] < pol["projected_ms"]["8"]
    # BERT-Large-sized gradients (1.34 GB) with a cap that only reaches 20 GB/s: 8 CTAs cannot
    # hide them in a 120 ms backward -> RCCL's default
    slow_cap = {8: _probe(0.05, 2.94, w), 0: _probe(0.025, 0.195, w)}
    big = [32 << 20] * 42
    pol = rccl.choose_cta_budget(slow_cap, big, w, overlap_ms=120.0)
    assert pol["cta_budget"] == 0 and "RCCL default" in pol["reason"]
    assert pol["projected_ms"]["8"] * 1.5 > 120.0
    # the same probes with the small ResNet gradients: 105 MB at 20 GB/s is ~9 ms, x1.5 < 44
    assert rccl.choose_cta_budget(slow_cap, buckets, w, overlap_ms=44.0)["cta_budget"] == 8
    # no overlap estimate: bandwidth ratio (50 % < 70 % -> default; 90 % -> cap)
    assert rccl.choose_cta_budget(fast, buckets, w)["cta_budget"] == 0
    near = {8: _probe(0.03, 0.217, w), 0: _probe(0.025, 0.195, w)}
    assert rccl.choose_cta_budget(near, buckets, w)["cta_budget"] == 8
    # one budget missing from the table: take the one that was measured
    assert rccl.choose_cta_budget({0: fast[0]}, buckets, w, overlap_ms=44.0)["cta_budget"] == 0
    assert rccl.choose_cta_budget({8: fast[8]}, buckets, w, overlap_ms=44.0)["cta_budget"] == 8


def test_cta_policy_latency_bound_small_buckets_raise_the_first_bucket():
    """A 1 MB all-reduce at < 25 % of the 32 MB bus bandwidth is latency-bound: the policy asks
    for an 8 MB first bucket, and BucketedAllReducer re-buckets with it."""
    from tensorflow_train_distributed_amd.parallel import collective, rccl
    from tensorflow_train_distributed_amd.train.flat import FlatParams, ParamSpec
    w = 8
    lat = {8: _probe(0.2, 0.39, w), 0: _probe(0.2, 0.195, w)}  # 1 MB in 200 us: ~9 GB/s
    pol = rccl.choose_cta_budget(lat, [32 << 20] * 4, w, overlap_ms=44.0)
    assert pol["first_bucket_mb"] == 8.0
    ok = {8: _probe(0.012, 0.39, w), 0: _probe(0.01, 0.195, w)}
    assert rccl.choose_cta_budget(ok, [32 << 20] * 4, w, overlap_ms=44.0)["first_bucket_mb"] is None
    # latency term: 100 buckets of 1 MB cost ~100 x the per-collective latency
    t_small = rccl.projected_step_ms(lat[0], [1 << 20] * 100, w)
    assert t_small > 100 * 0.15

    class FakeComm:
        max_ctas = 0
        policy = pol

    specs = [ParamSpec("v%d" % i, (n,), None, True) for i, n in enumerate([600000] * 10)]
    p = FlatParams(specs, "cpu", compute_dtype=None)
    red = collective.BucketedAllReducer(p, bucket_mb=32.0, first_bucket_mb=2.0)
    first_before = red.buckets[0][1] - red.buckets[0][0]
    red.comm = FakeComm()
    fb = red.policy()["first_bucket_mb"]
    red.first_bucket_mb = fb
    red._make_buckets()
    assert (red.buckets[0][1] - red.buckets[0][0]) * 4 >= 8 << 20 > first_before * 4
    assert red.buckets[-1][1] == p.numel and all(a[1] == b[0] for a, b in zip(red.buckets, red.buckets[1:]))
