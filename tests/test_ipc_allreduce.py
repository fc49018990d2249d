"""Direct xGMI all-reduce kernels (csrc/kernels/ipc_allreduce.hip, parallel/ipc.py) vs an fp32
sum, on one GPU:

* one rank, self-mapped staging buffers (the whole one-/two-shot path with world = 1);
* 2 ranks of ONE process (engines linked by pointers, each rank's kernel on its own HIP stream,
  running concurrently): barriers, two-shot chunk exchange, fp32 and bf16, every rank
  bit-identical. (More in-process ranks need as many concurrently scheduled streams; with
  GPU_MAX_HW_QUEUES = 4 two streams can share a hardware queue, then the later rank's kernel
  waits behind a spinning one until the barrier's bounded spin gives up — measured with 3.);
* 2 processes on the same GPU through real IPC handles (hipIpcGetMemHandle / OpenMemHandle over
  a gloo rendezvous on 127.0.0.1), eager and replayed from a captured hipGraph (the epoch lives
  in device memory, so replays see fresh barrier epochs);
* the failure contract: a rank that skips a call (lost / stalled peer) makes the other rank's
  barrier time out; the bucket then holds NaN, never a partial or stale sum, the host-mapped
  error word surfaces as UnavailableError at the next check (no device sync), later calls of
  the dead engine poison without waiting, and the skipping rank's next call fails too.
Multi-GPU runs use the same kernels with peers on other devices (xGMI)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

MB = 1 << 20


_STREAMS = []


def _streams(n):
    """The SAME n streams for every in-process test: each new HIP stream takes the next hardware
    queue round-robin, and two ranks whose streams share a queue cannot run concurrently."""
    while len(_STREAMS) < n:
        _STREAMS.append(torch.cuda.Stream())
    return _STREAMS[:n]


def _inputs(world, n, dtype, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return [(torch.rand(n, generator=g) * 2 - 1).to(dtype) for _ in range(world)]


def test_one_rank_self_mapped():
    from tensorflow_train_distributed_amd.parallel import ipc
    r = ipc.IpcAllReducer(device="cuda:0", cap_bytes=8 * MB)
    try:
        for path, n in [(ipc.ONE_SHOT, 4096), (ipc.TWO_SHOT, 3 * MB // 4)]:
            x = _inputs(1, n, torch.float32, n)[0].cuda()
            want = x.clone()
            r.all_reduce_(x, path)
            torch.cuda.synchronize()
            assert torch.equal(x, want)
        assert not r.timed_out()
    finally:
        r.destroy()


@pytest.mark.parametrize("world", [2])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_local_group_sum_vs_fp32(world, dtype):
    from tensorflow_train_distributed_amd.parallel import ipc
    grp = ipc.LocalGroup(world, device="cuda:0", cap_bytes=8 * MB)
    streams = _streams(world)
    try:
        esz = 4 if dtype == torch.float32 else 2
        for path, nbytes in [(ipc.ONE_SHOT, 64 * 1024), (ipc.ONE_SHOT, MB), (ipc.TWO_SHOT, 3 * MB + 1024),
                             (ipc.TWO_SHOT, 8 * MB)]:
            n = nbytes // esz
            xs = _inputs(world, n, dtype, nbytes + world)
            want = sum(x.float() for x in xs)
            dev = [x.cuda() for x in xs]
            torch.cuda.synchronize()
            for r in range(world):  # every rank's kernel on its own stream: they run concurrently
                grp.all_reduce_(r, dev[r], path, streams[r])
            torch.cuda.synchronize()
            assert not grp.timed_out(), "a barrier timed out (ranks did not run concurrently?)"
            for r in range(world):
                tol = 1e-6 if dtype == torch.float32 else 1e-2
                assert ((dev[r].float().cpu() - want).norm() / want.norm()).item() < tol
                assert torch.equal(dev[r], dev[0])
    finally:
        grp.destroy()


def _two_proc_worker(rank, world, port, q):
    try:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from tensorflow_train_distributed_amd.parallel import ipc
        r = ipc.IpcAllReducer(device="cuda:0", cap_bytes=8 * MB)
        res = {}
        for path, nbytes in [(ipc.ONE_SHOT, 256 * 1024), (ipc.TWO_SHOT, 5 * MB)]:
            n = nbytes // 4
            xs = _inputs(world, n, torch.float32, nbytes)
            want = sum(xs)
            x = xs[rank].cuda()
            r.all_reduce_(x, path)
            torch.cuda.synchronize()
            res[path] = ((x.cpu() - want).norm() / want.norm()).item()
        # captured once, replayed with fresh inputs (device-side epochs)
        n = 2 * MB // 4
        buf = torch.zeros(n, device="cuda")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            r.all_reduce_(buf, ipc.TWO_SHOT)
        errs = []
        for it in range(3):
            xs = _inputs(world, n, torch.float32, 77 + it)
            buf.copy_(xs[rank].cuda())
            dist.barrier()
            g.replay()
            torch.cuda.synchronize()
            want = sum(xs)
            errs.append(((buf.cpu() - want).norm() / want.norm()).item())
        res["replay"] = max(errs)
        res["timed_out"] = r.timed_out()
        r.destroy()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:  # noqa: BLE001 - reported to the test
        q.put((rank, "%s: %s" % (type(e).__name__, e)))


def test_two_processes_one_gpu_ipc():
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_two_proc_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(2):
            rank, res = q.get(timeout=100)
            out[rank] = res
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank in range(2):
        res = out[rank]
        assert isinstance(res, dict), res
        assert not res["timed_out"]
        for k, v in res.items():
            if k != "timed_out":
                assert v < 1e-6, (rank, k, v)


SPIN = 1 << 14  # barrier polls before a peer counts as lost: ~ms instead of the default ~1-2 s


@pytest.mark.parametrize("path", ["one", "two"])
def test_local_group_missing_peer_poisons_not_sums(path):
    from tensorflow_train_distributed_amd.parallel import ipc
    p = ipc.ONE_SHOT if path == "one" else ipc.TWO_SHOT
    grp = ipc.LocalGroup(2, device="cuda:0", cap_bytes=8 * MB, spin=SPIN)
    streams = _streams(2)
    try:
        n = (256 * 1024 if path == "one" else 3 * MB) // 4
        x = torch.ones(n, device="cuda")
        torch.cuda.synchronize()
        grp.all_reduce_(0, x, p, streams[0])  # rank 1 never calls
        torch.cuda.synchronize()
        assert grp.timed_out()
        assert bool(torch.isnan(x).all()), "a rank whose peer is missing must not return a sum"
        # the engine is dead: the next call poisons at once (no spin on the rank that failed)
        y = torch.ones(n, device="cuda")
        grp.all_reduce_(0, y, p, streams[0])
        torch.cuda.synchronize()
        assert bool(torch.isnan(y).all())
        grp.clear_error()
        assert not grp.timed_out()
    finally:
        grp.destroy()


def test_limited_blocks_sum_exact():
    """max_blocks (the collectives' CTA budget) caps the launch; the sum stays exact."""
    from tensorflow_train_distributed_amd.parallel import ipc
    grp = ipc.LocalGroup(2, device="cuda:0", cap_bytes=8 * MB, max_blocks=4)
    streams = _streams(2)
    try:
        for p, nbytes in [(ipc.ONE_SHOT, MB), (ipc.TWO_SHOT, 6 * MB)]:
            xs = _inputs(2, nbytes // 4, torch.float32, nbytes)
            dev = [x.cuda() for x in xs]
            torch.cuda.synchronize()
            for r in range(2):
                grp.all_reduce_(r, dev[r], p, streams[r])
            torch.cuda.synchronize()
            assert not grp.timed_out()
            want = xs[0] + xs[1]
            for r in range(2):
                assert torch.equal(dev[r].cpu(), want)
    finally:
        grp.destroy()


def _skip_worker(rank, world, port, q):
    try:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from tensorflow_train_distributed_amd.parallel import ipc
        from tensorflow_train_distributed_amd.utils import errors
        r = ipc.IpcAllReducer(device="cuda:0", cap_bytes=8 * MB, spin=SPIN)
        res = {}
        n = 512 * 1024 // 4
        # step 1: both ranks, exact
        x = torch.full((n,), float(rank + 1), device="cuda")
        r.all_reduce_(x, ipc.ONE_SHOT)
        torch.cuda.synchronize()
        res["step1_exact"] = bool((x == 3.0).all())
        r.check()
        dist.barrier()
        # step 2: rank 1 skips its call (a stalled / lost peer)
        x = torch.full((n,), float(rank + 1), device="cuda")
        if rank == 0:
            r.all_reduce_(x, ipc.ONE_SHOT)
        torch.cuda.synchronize()
        res["step2_nan"] = bool(torch.isnan(x).all()) if rank == 0 else None
        try:
            r.check()
            res["step2_raised"] = False
        except errors.UnavailableError:
            res["step2_raised"] = True
        dist.barrier()
        # step 3: both call again; rank 0's engine is dead (publishes nothing), so rank 1's
        # barrier times out too: the failure reaches the rank that skipped within one step
        x = torch.full((n,), float(rank + 1), device="cuda")
        r.all_reduce_(x, ipc.ONE_SHOT)
        torch.cuda.synchronize()
        res["step3_nan"] = bool(torch.isnan(x).all())
        try:
            r.check()
            res["step3_raised"] = False
        except errors.UnavailableError:
            res["step3_raised"] = True
        dist.barrier()
        r.destroy()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:  # noqa: BLE001 - reported to the test
        q.put((rank, "%s: %s" % (type(e).__name__, e)))


def test_two_processes_skipped_call_surfaces_error():
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_skip_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(2):
            rank, res = q.get(timeout=100)
            out[rank] = res
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank in range(2):
        assert isinstance(out[rank], dict), out[rank]
        assert out[rank]["step1_exact"]
    assert out[0]["step2_nan"] and out[0]["step2_raised"], out[0]
    assert not out[1]["step2_raised"], out[1]
    # no wrong sum is ever consumed: each rank's step-3 bucket is NaN and its check raises
    for rank in range(2):
        assert out[rank]["step3_nan"] and out[rank]["step3_raised"], (rank, out[rank])
