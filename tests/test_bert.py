"""BERT pre-training model: parameter inventory (CPU) and the GPU engine vs an fp32 PyTorch
reference of the same network (dropout off), plus a dropout-on training smoke."""
import pytest
import torch

from tensorflow_train_distributed_amd.models.bert import BertConfig, BertPretraining, synthetic_batch


def test_bert_large_parameter_inventory():
    cfg = BertConfig.large()
    # Google's BERT-Large (uncased, 24x1024x16) pre-training checkpoint incl. MLM/NSP heads
    assert BertPretraining.count_parameters(cfg) == 336226108
    specs = {s.name: s for s in BertPretraining.build_specs(cfg)}
    assert specs["bert/encoder/layer_23/attention/self/query/kernel"].meta["tf_shape"] == (1024, 1024)
    assert specs["bert/encoder/layer_0/intermediate/dense/kernel"].shape == (4096, 1024)
    assert specs["bert/embeddings/word_embeddings"].shape == (30528, 1024)
    names = [s.name for s in BertPretraining.build_specs(cfg)]
    # backward-completion layout: heads first, tied word embedding last
    assert names[0] == "cls/predictions/output_bias" and names[-1] == "bert/embeddings/word_embeddings"
    assert names.index("bert/encoder/layer_23/output/LayerNorm/gamma") < names.index(
        "bert/encoder/layer_0/output/LayerNorm/gamma")
    assert BertPretraining.count_parameters(BertConfig.base()) == 110106428


def test_bert_checkpoint_export_tf_layout(tmp_path):
    from tensorflow_train_distributed_amd.train import checkpoint as C
    cfg = BertConfig(vocab_size=1000, hidden_size=128, num_hidden_layers=1, num_attention_heads=2,
                     intermediate_size=256, max_position_embeddings=128)
    m = BertPretraining(cfg, device="cpu", seed=1)
    saver = C.Saver(m.params)
    path = saver.save(None, str(tmp_path / "model.ckpt"), global_step=3)
    shapes = dict(C.list_variables(path))
    assert shapes["bert/embeddings/word_embeddings"] == (1000, 128)
    assert shapes["cls/predictions/output_bias"] == (1000,)
    assert shapes["bert/encoder/layer_0/intermediate/dense/kernel"] == (128, 256)
    k = C.load_variable(path, "bert/encoder/layer_0/intermediate/dense/kernel")
    torch.testing.assert_close(torch.from_numpy(k), m.params.var["bert/encoder/layer_0/intermediate/dense/kernel"].t())
    m2 = BertPretraining(cfg, device="cpu", seed=2)
    C.Saver(m2.params).restore(None, path)
    assert torch.equal(m2.params.master, m.params.master)


@pytest.mark.gpu
@pytest.mark.parametrize("full_length", [True, False])
@pytest.mark.parametrize("gemms", ["own", "vendor_ab"])
def test_bert_engine_matches_reference(full_length, gemms):
    """gemms="own": every GEMM on our kernels (the product default: the 4-wave AGPR kernel for
    the K-major dense layers, the 256-row kernel for the rest); "vendor_ab": the hipBLASLt A/B
    mode (TTD_BERT_BLASLT=2), kept as an oracle path."""
    torch.manual_seed(0)
    cfg = BertConfig(vocab_size=1000, hidden_size=512, num_hidden_layers=2, num_attention_heads=8,
                     intermediate_size=1024, max_position_embeddings=256)
    m = BertPretraining(cfg, device="cuda", seed=3, dropout=False)
    m.blaslt = 0 if gemms == "own" else 2
    batch = synthetic_batch(cfg, 2, 256, max_predictions=20, device="cuda", seed=1, full_length=full_length)
    sums = m.forward_backward(batch)
    torch.cuda.synchronize()
    P = m.params
    leaves = {n: P.c[n].float().detach().clone().requires_grad_(True) for n in P.names()}
    for n in P.names():  # fp32 params used directly by the kernels (biases, LayerNorm)
        if n.endswith("/bias") or "LayerNorm" in n or n.endswith("output_bias"):
            leaves[n] = P.var[n].detach().clone().requires_grad_(True)
    mlm, nsp = m.reference_loss(batch, leaves)
    assert abs(float(sums[0]) - float(mlm)) < 0.02 * float(mlm), (float(sums[0]), float(mlm.detach()))
    assert abs(float(sums[2]) - float(nsp)) < 0.02 * float(nsp) + 1e-3
    (mlm + nsp).backward()
    ge, gr = [], []
    bad = []
    for n in P.names():
        a = P.g[n].flatten()
        b = leaves[n].grad
        b = torch.zeros_like(a) if b is None else b.flatten()
        if "rows" in P.spec(n).meta:  # padded vocab rows: must be exactly zero
            rows = P.spec(n).meta["rows"]
            width = a.numel() // P.spec(n).shape[0]
            assert float(a[rows * width:].abs().sum()) == 0.0, n
        ge.append(a)
        gr.append(b)
        if n.endswith("key/bias"):
            # softmax is invariant to q.b_k (constant over keys): the exact gradient is 0, the
            # engine's is bf16 rounding noise -- check it is small next to the query bias grad
            qn = float(P.g[n.replace("key/bias", "query/bias")].norm())
            assert float(a.norm()) < 0.05 * qn, (n, float(a.norm()), qn)
        elif b.norm() > 0:
            rel = float((a - b).norm() / b.norm())
            if rel > 0.1:
                bad.append((n, rel))
    ge, gr = torch.cat(ge), torch.cat(gr)
    cos = float(torch.dot(ge, gr) / (ge.norm() * gr.norm()))
    assert cos > 0.99, (cos, bad[:10])
    assert not bad, bad[:10]


@pytest.mark.gpu
def test_bert_training_with_dropout_lamb_decreases_loss():
    from tensorflow_train_distributed_amd.train.flat import FlatLAMB, Schedule
    torch.manual_seed(0)
    cfg = BertConfig(vocab_size=1000, hidden_size=512, num_hidden_layers=2, num_attention_heads=8,
                     intermediate_size=1024, max_position_embeddings=128)
    m = BertPretraining(cfg, device="cuda", seed=4)
    opt = FlatLAMB(m.params, Schedule(kind=0, base_lr=2e-3), weight_decay=0.01)
    batch = synthetic_batch(cfg, 4, 128, max_predictions=20, device="cuda", seed=2)
    losses = []
    for _ in range(30):
        s = m.forward_backward(batch)
        opt.step()
        losses.append(float(s[0]))
    assert all(l == l for l in losses)
    assert losses[-1] < losses[0] - 1.0, losses


@pytest.mark.gpu
def test_bert_step_segmented_capture_matches_eager():
    """The BERT step (side-stream weight gradients and transposed-weight refresh) recorded as
    per-stream graph segments replays the eager steps."""
    from tensorflow_train_distributed_amd.train.flat import FlatLAMB, Schedule
    from tensorflow_train_distributed_amd.utils import graphs
    cfg = BertConfig(vocab_size=1000, hidden_size=512, num_hidden_layers=2, num_attention_heads=8,
                     intermediate_size=1024, max_position_embeddings=128)
    batch = synthetic_batch(cfg, 4, 128, max_predictions=20, device="cuda", seed=2)

    def make():
        m = BertPretraining(cfg, device="cuda", seed=4, dropout=False)
        return m, FlatLAMB(m.params, Schedule(kind=0, base_lr=1e-3), weight_decay=0.01)

    m1, o1 = make()
    m2, o2 = make()
    assert m2.wgrad_stream

    def step(m, o):
        s = m.forward_backward(batch)
        o.step()
        return s

    eager = [step(m1, o1).clone() for _ in range(4)]
    main = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1])
    seg = graphs.capture_segmented(lambda: step(m2, o2), main=main, warmup=1)
    assert seg.info["streams"] == 2, seg.info
    replays = [seg.replay().clone() for _ in range(3)]
    torch.cuda.synchronize()
    for a, b in zip(eager[1:], replays):
        torch.testing.assert_close(a, b, rtol=3e-3, atol=3e-3)
    d = (m1.params.master - m2.params.master).abs().max()
    assert float(d) < 1e-3 * float(m1.params.master.abs().max()), float(d)
