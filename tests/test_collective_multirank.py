"""Multi-rank tests of the data-parallel gradient path on gloo (CPU): the bucketed all-reduce
(BucketedAllReducer) with distinct per-rank gradients, the mean-equals-big-batch property of
MirroredStrategy-style data parallelism on the reference MLP, and `bench.py --gpus N`
launching its own N ranks (the path the driver's scaling run uses, here over gloo).

Reference behaviour: synchronous aggregation applies the MEAN of the replicas' gradients
(/root/reference/distribute_training.py:142-152 via SyncReplicasOptimizer; the Mirrored
strategies of BASELINE.json do it by all-reduce).
"""
import json
import os
import subprocess
import sys

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _by_value(d):
    """Tensors -> numpy for the result queue: a tensor is shared by file descriptor, which races
    with the worker's exit (EOFError in the parent); numpy arrays are pickled by value."""
    return {k: (v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else v) for k, v in d.items()}


def _as_tensors(d):
    import numpy as np
    return {k: (torch.from_numpy(v) if isinstance(v, np.ndarray) else v) for k, v in d.items()}


def _spawn(fn, world, tmp_path, *args):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=fn, args=(r, world, str(tmp_path / "store"), q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return sorted((_as_tensors(r) for r in res), key=lambda r: r["rank"])


def _reducer_worker(rank, world, store, q, compress, algorithm="allreduce", num_packs=None):
    torch.set_num_threads(1)
    import torch.distributed as dist
    from tensorflow_train_distributed_amd.parallel.collective import BucketedAllReducer
    from tensorflow_train_distributed_amd.train.flat import FlatParams, ParamSpec
    dist.init_process_group("gloo", store=dist.FileStore(store, world), rank=rank, world_size=world)
    # variables in backward-completion order; sizes so that several buckets form
    specs = [ParamSpec("v%d" % i, (n,), None, True) for i, n in enumerate([20000, 3, 120000, 5000, 250000, 17])]
    p = FlatParams(specs, "cpu", compute_dtype=None)
    red = BucketedAllReducer(p, bucket_mb=0.6, first_bucket_mb=0.2, compress_bf16=compress, algorithm=algorithm,
                             num_packs=num_packs)
    g = torch.Generator().manual_seed(100 + rank)
    # each rank's gradient, pre-scaled by 1/world (zero in the alignment padding between variables)
    local = torch.randn(p.numel, generator=g) / world * p.valid_mask()
    red.begin()
    order = []
    for s in specs:  # backward: variables become final front to back
        o, n = p.offsets[s.name], s.shape[0]
        p.grad[o:o + n] = local[o:o + n]
        red.mark_ready(s.name)
        order.append(list(red.launch_log))
    red.finish()
    q.put(_by_value({"rank": rank, "grad": p.grad.clone(), "local": local, "buckets": red.buckets,
           "log": red.launch_log, "order": order, "bytes": red.bytes_per_step()}))
    dist.destroy_process_group()


@pytest.mark.parametrize("compress", [False, True])
def test_bucketed_allreduce_mean_and_order(tmp_path, compress):
    world = 3
    res = _spawn(_reducer_worker, world, tmp_path, compress)
    buckets = res[0]["buckets"]
    assert len(buckets) >= 3
    # buckets are contiguous, cover the buffer, launched in order as soon as their last
    # variable is final (not all at finish())
    assert buckets[0][0] == 0 and all(a[1] == b[0] for a, b in zip(buckets, buckets[1:]))
    assert res[0]["log"] == list(range(len(buckets)))
    assert len(res[0]["order"][0]) == 0 and len(res[0]["order"][-1]) == len(buckets)
    assert 0 < len(res[0]["order"][2]) < len(buckets)
    mean = sum(r["local"] for r in res)  # sum of the 1/world-scaled gradients == mean
    for r in res:
        if compress:
            torch.testing.assert_close(r["grad"], mean, rtol=2e-2, atol=1e-2)  # bf16 on the wire and in the sum
        else:
            torch.testing.assert_close(r["grad"], mean, rtol=1e-6, atol=1e-7)
        if not compress:  # every replica holds the same result (gloo's bf16 sums may round per rank)
            assert torch.equal(r["grad"], res[0]["grad"])
    assert res[0]["bytes"] == buckets[-1][1] * (2 if compress else 4)


@pytest.mark.parametrize("algorithm,num_packs", [("hierarchical", None), ("reduce_to_one", None),
                                                 ("allreduce", 2), ("hierarchical", 3)])
def test_cross_device_ops_algorithms_give_the_mean(tmp_path, algorithm, num_packs):
    """HierarchicalCopyAllReduce (reduce-scatter + all-gather, ragged buckets padded),
    ReductionToOneDevice (reduce to rank 0 + broadcast) and RcclAllReduce(num_packs=k)."""
    world = 3
    res = _spawn(_reducer_worker, world, tmp_path, False, algorithm, num_packs)
    buckets = res[0]["buckets"]
    if num_packs:
        assert len(buckets) == num_packs
    mean = sum(r["local"] for r in res)
    for r in res:
        torch.testing.assert_close(r["grad"], mean, rtol=1e-6, atol=1e-7)
        assert torch.equal(r["grad"], res[0]["grad"])


def test_strategy_cross_device_ops_classes_select_algorithms():
    from tensorflow_train_distributed_amd.parallel import strategy as S
    assert S.HierarchicalCopyAllReduce(num_packs=2).algorithm == "hierarchical"
    assert S.ReductionToOneDevice().algorithm == "reduce_to_one"
    assert S.NcclAllReduce is S.RcclAllReduce and S.RcclAllReduce(num_packs=4).num_packs == 4


def _mlp_worker(rank, world, store, q):
    torch.set_num_threads(1)
    import torch.distributed as dist
    from tensorflow_train_distributed_amd.models.mlp import mnist_mlp
    from tensorflow_train_distributed_amd.parallel.collective import BucketedAllReducer, broadcast_flat_
    dist.init_process_group("gloo", store=dist.FileStore(store, world), rank=rank, world_size=world)
    model = mnist_mlp(device="cpu", seed=11 + rank, dropout_rate=0.0)  # differently initialised replicas
    broadcast_flat_(model.params)
    red = BucketedAllReducer(model.params, bucket_mb=0.25, first_bucket_mb=0.1)
    g = torch.Generator().manual_seed(5)
    B = 32
    x = torch.rand((B * world, 784), generator=g)
    y = torch.randint(0, 10, (B * world,), generator=g)
    red.begin()
    model.forward_backward({"x-input": x[rank * B:(rank + 1) * B], "y-input": y[rank * B:(rank + 1) * B]},
                           grad_scale=1.0 / (B * world), grad_hook=red.mark_ready)
    red.finish()
    dp = model.params.grad.clone()
    # the same step on one replica holding the whole global batch
    model.forward_backward({"x-input": x, "y-input": y})
    q.put(_by_value({"rank": rank, "dp": dp, "big": model.params.grad.clone(), "w": model.params.master.clone()}))
    dist.destroy_process_group()


def test_mirrored_gradient_equals_big_batch_gradient(tmp_path):
    res = _spawn(_mlp_worker, 2, tmp_path)
    assert torch.equal(res[0]["w"], res[1]["w"])  # broadcast synchronised the replicas
    for r in res:
        torch.testing.assert_close(r["dp"], r["big"], rtol=2e-5, atol=2e-6)


@pytest.mark.slow
@pytest.mark.parametrize("n", [2, 4])
def test_bench_self_launches_n_ranks(n):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["CUDA_VISIBLE_DEVICES"] = ""
    p = subprocess.run([sys.executable, "bench.py", "--model", "mlp", "--device", "cpu", "--gpus", str(n),
                        "--steps", "3", "--warmup", "1"], cwd=REPO, env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # one JSON line, from rank 0
    r = json.loads(lines[0])
    assert r["n_gpus"] == n and r["dist"]["world_size"] == n and r["dist"]["backend"] == "gloo"
    assert r["dist"]["replicas_in_sync"] is True and len(r["dist"]["per_rank_ms"]) == n
    assert r["config"]["global_batch"] == 128 * n
    assert r["dist"]["allreduce_bytes_per_step"] >= 183685 * 4
    assert r["value"] > 0 and r["ms_per_step"] > 0


def _tape_worker(rank, world, store, q, clip=None):
    """tf.distribute custom training loop on a user-defined ttd.layers model: GradientTape +
    optimizer.apply_gradients inside strategy.run, replicas on gloo."""
    torch.set_num_threads(1)
    import torch.distributed as dist
    import tensorflow_train_distributed_amd as ttd
    from tensorflow_train_distributed_amd.parallel import strategy as S
    dist.init_process_group("gloo", store=dist.FileStore(store, world), rank=rank, world_size=world)
    strategy = S.Strategy("cpu")
    ttd.layers.reset_naming(seed=100 + rank)  # replicas start from different weights
    with strategy.scope():
        model = ttd.layers.Sequential([ttd.layers.Dense(32, activation="relu"), ttd.layers.Dense(10)])
        opt = ttd.train.MomentumOptimizer(0.1, 0.9)
    g = torch.Generator().manual_seed(3)
    B = 16
    X = torch.randn(4, B * world, 20, generator=g)
    Y = torch.randint(0, 10, (4, B * world), generator=g)
    losses = []

    def step_fn(x, y):
        with ttd.GradientTape() as tape:
            logits = model(x)
            loss = torch.nn.functional.cross_entropy(logits, y, reduction="sum") / (B * world)
        grads = tape.gradient(loss, model.trainable_variables)
        if clip is not None:  # the caller rewrites the gradients before applying them
            grads, _ = ttd.clip_by_global_norm(grads, clip)
        opt.apply_gradients(zip(grads, model.trainable_variables))
        return loss

    for i in range(4):
        xs, ys = X[i, rank * B:(rank + 1) * B], Y[i, rank * B:(rank + 1) * B]
        losses.append(float(strategy.reduce(S.ReduceOp.SUM, strategy.run(step_fn, args=(xs, ys)))))
    q.put(_by_value({"rank": rank, "w": model.params.master.clone(), "names": model.params.names(), "losses": losses,
           "X": X, "Y": Y, "init": getattr(model, "_ttd_init", None)}))
    dist.destroy_process_group()


@pytest.mark.parametrize("clip", [None, 0.05, 1e9])
def test_gradient_tape_apply_gradients_matches_big_batch(tmp_path, clip):
    """clip: gradients clipped (0.05: every step clips) or rescaled by exactly 1 (1e9) between
    tape.gradient and apply_gradients -- they must not be all-reduced a second time."""
    import tensorflow_train_distributed_amd as ttd
    res = _spawn(_tape_worker, 2, tmp_path, clip)
    assert torch.equal(res[0]["w"], res[1]["w"])  # replicas identical (rank 0's init was broadcast)
    # the same 4 steps in one process over the whole global batch, from rank 0's initial weights
    ttd.layers.reset_naming(seed=100)
    model = ttd.layers.Sequential([ttd.layers.Dense(32, activation="relu"), ttd.layers.Dense(10)])
    model(res[0]["X"][0, :1])
    flat = model.to_flat("cpu")
    opt = ttd.train.MomentumOptimizer(0.1, 0.9)
    X, Y = res[0]["X"], res[0]["Y"]
    for i in range(4):
        with ttd.GradientTape() as tape:
            loss = torch.nn.functional.cross_entropy(model(X[i]), Y[i])
        grads = tape.gradient(loss, model.trainable_variables)
        if clip is not None:
            grads, _ = ttd.clip_by_global_norm(grads, clip)
        opt.apply_gradients(zip(grads, model.trainable_variables))
    assert flat.names() == res[0]["names"]
    torch.testing.assert_close(res[0]["w"], flat.master, rtol=2e-5, atol=2e-5)


class _FakeComm:
    """Stands in for RcclCommunicator in the CTA-budget probe: fixed probe times per budget,
    optional failure at a chosen budget."""

    def __init__(self, ctas, fail, ms):
        if fail:
            raise RuntimeError("injected communicator failure (budget %d)" % ctas)
        self.max_ctas, self.ms, self.destroyed = ctas, ms, None

    def probe(self, nbytes, iters=5):
        return {"bytes": int(nbytes), "ms": self.ms * (1 + nbytes / (64 << 20)), "busbw_GBps": 0.0}

    def destroy(self, abort=False):
        self.destroyed = "abort" if abort else "finalize"


def _probe_worker(rank, world, store, q, fail_rank, fail_budget):
    torch.set_num_threads(1)
    import torch.distributed as dist
    from tensorflow_train_distributed_amd.parallel import rccl
    dist.init_process_group("gloo", store=dist.FileStore(store, world), rank=rank, world_size=world)
    rccl.unique_id = lambda: bytes(range(128))  # no RCCL on the CPU: any 128 bytes
    made = []

    def make(uid, w, r, dev, ctas):
        c = _FakeComm(ctas, r == fail_rank and ctas == fail_budget, ms=1.0 + 0.1 * r + (0.5 if ctas else 0.0))
        made.append(c)
        return c

    out = {"rank": rank}
    try:
        comm = rccl._probe_budgets(None, 40.0, [8 << 20, 32 << 20], make=make)
        out["budget"] = comm.policy["cta_budget"]
        out["ms"] = [d["ms"] for d in comm.policy["probe"][comm.policy["cta_budget"]]] \
            if isinstance(comm.policy.get("probe"), dict) else None
    except Exception as e:  # noqa: BLE001 - reported to the parent
        out["error"] = "%s: %s" % (type(e).__name__, e)
    out["destroyed"] = [c.destroyed for c in made]
    # the process group must still be in step: one more collective completes on every rank
    t = torch.ones(1)
    dist.all_reduce(t)
    out["after"] = float(t.item())
    q.put(out)
    dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank,fail_budget", [(None, None), (1, 0), (0, 8)])
def test_cta_budget_probe_failure_on_one_rank_fails_every_rank_together(tmp_path, fail_rank, fail_budget):
    """a communicator / probe failure on one rank must not leave the ranks in
    different torch collectives. Every rank joins the same id broadcast and the same MAX
    all-reduce (slot 0 = failure flag), then all raise together, or all pick the same budget."""
    world = 3
    res = _spawn(_probe_worker, world, tmp_path, fail_rank, fail_budget)
    assert all(r["after"] == world for r in res)  # the group is still usable afterwards
    if fail_rank is None:
        assert len({r["budget"] for r in res}) == 1 and all("error" not in r for r in res)
    else:
        assert all("error" in r and "UnavailableError" in r["error"] for r in res), res
        assert "this rank" in res[fail_rank]["error"]
        assert all("another rank" in r["error"] for i, r in enumerate(res) if i != fail_rank)
        # every communicator a rank did create is aborted
        assert all(all(d == "abort" for d in r["destroyed"] if d is not None) for r in res)
