"""Plan of the direct xGMI all-reduce (csrc/kernels/ipc_plan.h through libttd_rt.so): the
per-bucket path choice and the rank-chunk / workgroup-part partition the one-shot / two-shot
kernels (ipc_allreduce.hip) rely on, checked on the CPU for 2..8 ranks — including a NumPy
replay of the two-shot algorithm with per-workgroup barriers, which shows that each workgroup's
barrier covers exactly the data its peers' workgroups read."""
import numpy as np
import pytest

from tensorflow_train_distributed_amd.parallel import ipc

MB = 1 << 20


def test_choose_paths():
    cap = 8 * MB
    assert ipc.choose(4096, 8, True, cap) == ipc.ONE_SHOT
    assert ipc.choose(MB, 8, True, cap) == ipc.ONE_SHOT
    assert ipc.choose(MB + 16, 8, True, cap) == ipc.TWO_SHOT
    assert ipc.choose(8 * MB, 8, True, cap) == ipc.TWO_SHOT
    assert ipc.choose(8 * MB + 16, 8, True, cap) == ipc.RCCL
    assert ipc.choose(32 * MB, 8, True, cap) == ipc.RCCL
    assert ipc.choose(MB, 8, False, cap) == ipc.RCCL      # several nodes: peers not mappable
    assert ipc.choose(MB, 1, True, cap) == ipc.RCCL       # nothing to reduce
    assert ipc.choose(MB, 9, True, cap) == ipc.RCCL       # beyond one node's 8 GPUs
    assert ipc.choose(2 * MB, 8, True, MB) == ipc.RCCL    # larger than the staging buffers
    assert ipc.choose(0, 8, True, cap) == ipc.RCCL


def test_plan_paths_edges_only():
    b = [4 * MB, 32 * MB, 32 * MB, 512 * 1024]
    assert ipc.plan_paths(b, 8, True, 8 * MB) == [ipc.TWO_SHOT, ipc.RCCL, ipc.RCCL, ipc.ONE_SHOT]
    assert ipc.plan_paths(b, 8, False, 8 * MB) == [ipc.RCCL] * 4
    assert ipc.plan_paths([MB, MB, MB], 4, True, 8 * MB, edges_only=False) == [ipc.ONE_SHOT] * 3


@pytest.mark.parametrize("world", [2, 3, 4, 8])
@pytest.mark.parametrize("vec", [4, 8])
def test_chunks_and_parts_cover_exactly_once(world, vec):
    rng = np.random.default_rng(world * 10 + vec)
    for count in [vec, 2 * vec, 1000 * vec, int(rng.integers(1, 50000)) * vec]:
        cover = np.zeros(count, dtype=np.int32)
        prev = 0
        for r in range(world):
            lo, hi = ipc.chunk(count, vec, world, r)
            assert lo == prev and lo <= hi and lo % vec == 0 and hi % vec == 0
            prev = hi
            nb = ipc.blocks_for(count * 4)
            pprev = lo
            for b in range(nb):
                plo, phi = ipc.part(lo, hi, vec, nb, b)
                assert plo == pprev and plo <= phi and plo % vec == 0
                pprev = phi
                cover[plo:phi] += 1
            assert pprev == hi
        assert prev == count
        assert np.all(cover == 1)


@pytest.mark.parametrize("world", [2, 5, 8])
def test_two_shot_replay_with_per_block_barriers(world):
    """NumPy replay of the two-shot kernel: block b of every rank stages part b of every chunk,
    barrier(0, b), reduces part b of its own chunk from the peers' staged copies, barrier(1, b),
    gathers part b of every other chunk from that chunk's owner. Every read is asserted to fall
    in data the SAME block index wrote before its barrier on the peer."""
    vec = 4
    count = 4 * 3 * 1037
    rng = np.random.default_rng(world)
    x = rng.standard_normal((world, count)).astype(np.float32)
    nb = ipc.blocks_for(count * 4)
    staged = [np.full(count, np.nan, np.float32) for _ in range(world)]
    staged_by = [np.full(count, -1) for _ in range(world)]  # which block index staged each element
    out_reg = [np.full(count, np.nan, np.float32) for _ in range(world)]
    out_by = [np.full(count, -1) for _ in range(world)]
    result = [x[r].copy() for r in range(world)]
    for r in range(world):  # stage (before barrier 0)
        for b in range(nb):
            for q in range(world):
                lo, hi = ipc.part(*ipc.chunk(count, vec, world, q), vec, nb, b)
                staged[r][lo:hi] = x[r][lo:hi]
                staged_by[r][lo:hi] = b
    for r in range(world):  # reduce-scatter (after barrier 0, before barrier 1)
        for b in range(nb):
            lo, hi = ipc.part(*ipc.chunk(count, vec, world, r), vec, nb, b)
            acc = np.zeros(hi - lo, np.float32)
            for p in range(world):
                assert np.all(staged_by[p][lo:hi] == b)
                acc += staged[p][lo:hi]
            result[r][lo:hi] = acc
            out_reg[r][lo:hi] = acc
            out_by[r][lo:hi] = b
    for r in range(world):  # all-gather (after barrier 1)
        for b in range(nb):
            for q in range(world):
                if q == r:
                    continue
                lo, hi = ipc.part(*ipc.chunk(count, vec, world, q), vec, nb, b)
                assert np.all(out_by[q][lo:hi] == b)
                result[r][lo:hi] = out_reg[q][lo:hi]
    want = x.sum(0)
    for r in range(world):
        np.testing.assert_allclose(result[r], want, rtol=1e-5, atol=1e-5)
        assert np.array_equal(result[r], result[0])  # every rank holds the same bits


def test_reducer_bucket_paths_on_torch_backend():
    """On a non-native process group every bucket reports the torch backend."""
    import torch.distributed as dist
    from tensorflow_train_distributed_amd.parallel.collective import BucketedAllReducer
    if dist.is_initialized():
        pytest.skip("needs a fresh process")

    class _Flat:  # minimal FlatParams stand-in: two variables
        class _S:
            def __init__(self, name, shape):
                self.name, self.shape = name, shape
        specs = [_S("a", (1024,)), _S("b", (4096,))]
        offsets = {"a": 0, "b": 1024}
        numel = 5120

        class grad:  # noqa: N801
            is_cuda = False
    r = BucketedAllReducer(_Flat(), first_bucket_mb=0.001, bucket_mb=0.01)
    assert r.bucket_paths == ["none"] * len(r.buckets)


def test_blocks_for_respects_cta_budget():
    # ~16 KB per workgroup, 8 .. 64, and never above the collectives' CTA budget
    assert ipc.blocks_for(4096) == 8
    assert ipc.blocks_for(MB) == 64
    assert ipc.blocks_for(8 * MB) == 64
    for budget in (1, 4, 8, 16):
        for nbytes in (4096, 256 * 1024, MB, 8 * MB):
            assert ipc.blocks_for(nbytes, budget) == min(budget, ipc.blocks_for(nbytes))


def test_direct_path_is_opt_in(monkeypatch):
    monkeypatch.delenv("TTD_IPC_AR", raising=False)
    assert not ipc.enabled()
    monkeypatch.setenv("TTD_IPC_AR", "1")
    assert ipc.enabled()


def test_reducer_raises_when_direct_path_failed():
    """begin() / finish() surface the direct path's error word as UnavailableError (the
    session's recovery trigger) without a device sync."""
    from tensorflow_train_distributed_amd.parallel.collective import BucketedAllReducer
    from tensorflow_train_distributed_amd.utils import errors

    class FakeIpc:
        failed = False

        def check(self):
            if self.failed:
                raise errors.UnavailableError("peer lost")

    r = BucketedAllReducer.__new__(BucketedAllReducer)
    r.ipc = FakeIpc()
    r.begin()  # healthy: no raise
    r.ipc.failed = True
    with pytest.raises(errors.UnavailableError):
        r.begin()
