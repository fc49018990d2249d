"""BERT pre-training (masked-LM + next-sentence) on the gfx950 kernel library —
BASELINE.json config 4 ("BERT-Large seq=512 bf16 MirroredStrategy"), SURVEY.md §2.6 [NS]
BERT kernel list (embedding gather/scatter, LayerNorm, QKV/out-proj/FFN GEMMs, fused
attention, GELU, dropout, Adam/LAMB).

Execution model (MI355X-first, mirrors models/resnet.py):
* activations are token-major bf16 [B*S, features]; the fused QKV projection writes
  [tokens, 3H] and the attention kernels read Q/K/V as strided column slices of it and write
  dQ/dK/dV back into one [tokens, 3H] gradient, so no head transposes exist;
* dense kernels are stored [out, in] (the GEMM's K-major B operand; the checkpoint layer
  exports TF's [in, out]); q/k/v kernels and biases are adjacent in the flat store so the
  fused [3H, H] projection is a zero-copy view;
* every sub-layer epilogue is fused: bias (+GELU, keeping the pre-activation for backward)
  in the GEMM epilogue; residual add + hidden dropout + LayerNorm in one pass; GELU'
  multiplies inside the dgrad GEMM epilogue;
* dropout masks are counter hashes of a device-resident (seed, step) — nothing is stored,
  backward regenerates them, and a hipGraph-captured step still draws fresh masks;
* variables live in one FlatParams store in backward-completion order (heads, pooler,
  layers L-1..0, embeddings; the tied word embedding last) so bucketed all-reduce
  (parallel/collective.py) launches as soon as each layer's gradients are final;
* the vocabulary is padded to a multiple of 64 (zero rows, masked out of the softmax and
  sliced off in checkpoints) so the decoder GEMM and the vocab softmax stay vectorised.

Variable names follow Google's TF BERT checkpoints (bert/encoder/layer_N/attention/self/
query/kernel, cls/predictions/output_bias, ...).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from ..train.flat import FlatParams, ParamSpec
from ..utils import graphs


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 1024
    num_hidden_layers: int = 24
    num_attention_heads: int = 16
    intermediate_size: int = 4096
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    layer_norm_eps: float = 1e-12
    initializer_range: float = 0.02

    @property
    def vocab_padded(self) -> int:
        return (self.vocab_size + 63) // 64 * 64

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads

    @staticmethod
    def large(**kw) -> "BertConfig":
        return BertConfig(**kw)

    @staticmethod
    def base(**kw) -> "BertConfig":
        d = dict(hidden_size=768, num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072)
        d.update(kw)
        return BertConfig(**d)


def _trunc(std, rows=None):
    def init(t, gen):
        torch.nn.init.trunc_normal_(t, 0.0, std, -2 * std, 2 * std, generator=gen)
        if rows is not None:
            t[rows:] = 0.0
    init.dev = (1, 0.0, float(std))  # device init: truncated normal (init.hip)
    init.dev_zero_rows = rows
    return init


def _fill(v):
    def init(t, gen):
        t.fill_(v)
    init.dev = (3, float(v), 0.0)
    return init


@dataclass
class BertBatch:
    input_ids: torch.Tensor          # int32 [B, S]
    token_type_ids: torch.Tensor     # int32 [B, S]
    masked_lm_positions: torch.Tensor  # int32 [B, P] positions within the sequence
    masked_lm_ids: torch.Tensor      # int32 [B, P] (-1 = padding slot)
    next_sentence_labels: torch.Tensor  # int32 [B]
    seqlen: Optional[torch.Tensor] = None  # int32 [B] valid lengths (None = all S)


def synthetic_batch(cfg: BertConfig, B: int, S: int, max_predictions: int = 80, device="cuda", seed: int = 0,
                    full_length: bool = True) -> BertBatch:
    """Random-token pre-training batch of the shape of BERT's seq-512 phase-2 data
    (max_predictions_per_seq = 80): distinct masked positions, random targets."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    lo = min(1000, cfg.vocab_size // 2)  # skip BERT's [unused]/special-token id range
    ids = torch.randint(lo, cfg.vocab_size, (B, S), generator=g, dtype=torch.int32)
    tt = torch.zeros((B, S), dtype=torch.int32)
    half = torch.randint(S // 4, 3 * S // 4, (B,), generator=g)
    for b in range(B):
        tt[b, int(half[b]):] = 1
    pos = torch.stack([torch.randperm(S - 1, generator=g)[:max_predictions] + 1 for _ in range(B)]).sort(1).values
    lab = torch.randint(lo, cfg.vocab_size, (B, max_predictions), generator=g, dtype=torch.int32)
    nsp = torch.randint(0, 2, (B,), generator=g, dtype=torch.int32)
    seqlen = None
    if not full_length:
        seqlen = torch.randint(S // 2, S + 1, (B,), generator=g, dtype=torch.int32)
        for b in range(B):
            L = int(seqlen[b])
            keep = pos[b] < L
            lab[b][~keep] = -1
    return BertBatch(ids.to(device), tt.to(device), pos.to(torch.int32).to(device), lab.to(device), nsp.to(device),
                     seqlen.to(device) if seqlen is not None else None)


class BertPretraining:
    """BERT encoder + masked-LM / NSP heads with a hand-scheduled forward/backward."""

    def __init__(self, cfg: BertConfig, device="cuda", seed: int = 0, dropout: bool = True):
        if cfg.head_dim != 64:
            raise ValueError("the attention kernels are specialised for head_dim 64")
        self.cfg = cfg
        self.device = torch.device(device)
        self.dropout = dropout
        self.params = FlatParams(self.build_specs(cfg), self.device, seed=seed,
                                 device_init=os.environ.get("TTD_DEVICE_INIT", "1") != "0")
        P = self.params
        H, I, L = cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers
        for name_a, n, width in [("query/kernel", 3, H * H), ("query/bias", 3, H)]:
            for l in range(L):
                o = P.offsets[self._ln(l, "attention/self/" + name_a)]
                for j, nm in enumerate(["query", "key", "value"]):
                    o2 = P.offsets[self._ln(l, "attention/self/%s/%s" % (nm, name_a.split("/")[1]))]
                    if o2 != o + j * width:
                        raise AssertionError("q/k/v %s not contiguous" % name_a)
        self.rng = None
        # workgroups each side-stream weight-gradient GEMM aims for (split-K count): 192 of the 256
        # CUs leave room for the data-gradient chain's kernels (b128: 180.0 -> 176.8 ms/step over
        # two A/B pairs; 128: 177.4); TTD_BERT_WGRAD_WGS
        self.wgrad_wgs = int(os.environ.get("TTD_BERT_WGRAD_WGS", "192"))
        # side-stream weight gradients that would overlap a LayerNorm backward start after it
        # (TTD_BERT_LN_YIELD=0: as soon as their operands exist)
        # (2: also the attention backward)
        self.ln_yield = int(os.environ.get("TTD_BERT_LN_YIELD", "1"))
        # encoder weight gradients on a second HIP stream (TTD_WGRAD_STREAM=0: single stream)
        self.wgrad_stream = os.environ.get("TTD_WGRAD_STREAM", "1") != "0" and self.device.type == "cuda"
        # data-gradient GEMMs read [in][out] copies of the encoder weights (K-major B: ~10 % faster
        # than the MN-major [out][in] read); refreshed each step on the side stream during the
        # forward pass (TTD_BERT_WT=0: off)
        self.transposed_dgrad = os.environ.get("TTD_BERT_WT", "1") != "0" and self.device.type == "cuda"
        # FFN1 bias gradient from the dGELU dgrad epilogue column statistics instead of a colsum pass
        # on the side stream (TTD_BERT_BIAS_STAT=1; measured neutral-to-slower: 190.4 vs 188.5 ms)
        self.fuse_bias_grad = os.environ.get("TTD_BERT_BIAS_STAT", "0") != "0" and self.device.type == "cuda"
        # encoder bias gradients formed inside their weight-gradient GEMM from the dy tiles in LDS
        # (ops.gemm.gemm_wgrad_bias) instead of a column-sum pass over dy (TTD_BERT_BIAS_WGRAD=0: off)
        self.bias_in_wgrad = os.environ.get("TTD_BERT_BIAS_WGRAD", "1") != "0" and self.device.type == "cuda"
        # GEMM path. 0 (default): every GEMM on our kernels — the K-major dense layers (QKV,
        # attention output, FFN1 with bias + GELU + pre-activation store, FFN2, MLM logits, and the
        # data gradients on the [in][out] weight copies) on the 4-wave AGPR-accumulator kernel
        # (gemm4w.hip), the rest on the 256-row kernels. The vendor library (torch.addmm / mm ->
        # hipBLASLt) is an A/B and oracle mode only, TTD_BERT_BLASLT: 1 = the forward's bias-only
        # GEMMs, 2 = also the plain / accumulating data gradients, 3 = the weight gradients too.
        self.blaslt = int(os.environ.get("TTD_BERT_BLASLT", "0")) if self.device.type == "cuda" else 0
        # row-stride padding (elements) of the [tokens, intermediate] activations (FFN1 output, its
        # pre-activation, the dGELU gradient): with a power-of-two row stride (4096 x 2 B) every row
        # of a 256-row output tile falls on the same HBM channel group; measured on the FFN1 GEMM
        # (tools/g4_bench.py shapes): plain store 573 -> 482 us, bias + GELU + aux 640 -> 572 us
        # (stride 4352). TTD_BERT_IPAD=0: dense rows
        self.inter_pad = int(os.environ.get("TTD_BERT_IPAD", "256"))
        self._wt = None
        self._wt_batch = None
        # TTD_BERT_WT_BATCH=0: one transpose launch per weight copy instead of one batched launch
        self.wt_batch = os.environ.get("TTD_BERT_WT_BATCH", "1") != "0"
        if self.device.type == "cuda":
            from ..ops.transformer import RngState
            self.rng = RngState(seed * 7919 + 17, self.device)

    def _plain(self, x, w, b, b16):
        """y = x w^T + b (w [out][in] bf16; b fp32, b16 its bf16 compute copy) for the forward's
        bias-only GEMMs."""
        if self.blaslt:
            return torch.addmm(b16, x, w.t())
        from ..ops import gemm as G
        return G.gemm(x, w, trans_b=True, bias=b)

    # ------------------------------------------------------------------ variables
    @staticmethod
    def _ln(l, suffix):
        return "bert/encoder/layer_%d/%s" % (l, suffix)

    @staticmethod
    def build_specs(cfg: BertConfig) -> List[ParamSpec]:
        c = cfg
        H, I, V, Vp = c.hidden_size, c.intermediate_size, c.vocab_size, c.vocab_padded
        std = c.initializer_range
        sp: List[ParamSpec] = []

        def dense(name, n_out, n_in):
            sp.append(ParamSpec(name + "/kernel", (n_out, n_in), _trunc(std),
                                meta={"layout": "NK", "tf_shape": (n_in, n_out)}))

        def bias(name, n):
            sp.append(ParamSpec(name, (n,), _fill(0.0), weight_decay=False))

        def ln(name):
            sp.append(ParamSpec(name + "/gamma", (H,), _fill(1.0), weight_decay=False))
            sp.append(ParamSpec(name + "/beta", (H,), _fill(0.0), weight_decay=False))

        bias_spec = ParamSpec("cls/predictions/output_bias", (Vp,), _fill(0.0), weight_decay=False,
                              meta={"rows": V})
        sp.append(bias_spec)
        ln("cls/predictions/transform/LayerNorm")
        dense("cls/predictions/transform/dense", H, H)
        bias("cls/predictions/transform/dense/bias", H)
        # TF keeps output_weights as [2, H] = [out, in] already
        sp.append(ParamSpec("cls/seq_relationship/output_weights", (2, H), _trunc(std)))
        bias("cls/seq_relationship/output_bias", 2)
        dense("bert/pooler/dense", H, H)
        bias("bert/pooler/dense/bias", H)
        for l in reversed(range(c.num_hidden_layers)):
            p = lambda s, l=l: BertPretraining._ln(l, s)  # noqa: E731
            ln(p("output/LayerNorm"))
            dense(p("output/dense"), H, I)
            bias(p("output/dense/bias"), H)
            dense(p("intermediate/dense"), I, H)
            bias(p("intermediate/dense/bias"), I)
            ln(p("attention/output/LayerNorm"))
            dense(p("attention/output/dense"), H, H)
            bias(p("attention/output/dense/bias"), H)
            for nm in ("query", "key", "value"):
                dense(p("attention/self/" + nm), H, H)
            for nm in ("query", "key", "value"):
                bias(p("attention/self/%s/bias" % nm), H)
        ln("bert/embeddings/LayerNorm")
        sp.append(ParamSpec("bert/embeddings/token_type_embeddings", (c.type_vocab_size, H), _trunc(std)))
        sp.append(ParamSpec("bert/embeddings/position_embeddings", (c.max_position_embeddings, H), _trunc(std)))
        sp.append(ParamSpec("bert/embeddings/word_embeddings", (Vp, H), _trunc(std, rows=V), meta={"rows": V}))
        return sp

    @staticmethod
    def count_parameters(cfg: BertConfig) -> int:
        """Unpadded parameter count (what a TF checkpoint of this config holds)."""
        n = 0
        for s in BertPretraining.build_specs(cfg):
            shape = list(s.shape)
            if "rows" in s.meta:
                shape[0] = s.meta["rows"]
            n += int(np.prod(shape))
        return n

    _WT_NAMES = ("attention/output/dense/kernel", "intermediate/dense/kernel", "output/dense/kernel")

    def _refresh_transposed(self):
        """[in][out] copies of each layer's weights (fused QKV + the three dense kernels)."""
        from ..ops import kernels as K
        P, L = self.params, self.cfg.num_hidden_layers
        if self._wt is None:
            self._wt = []
            for l in range(L):
                ws = [self._fused(l, "w")] + [P.c[self._ln(l, n)] for n in self._WT_NAMES]
                self._wt.append([torch.empty((w.shape[1], w.shape[0]), dtype=w.dtype, device=w.device) for w in ws])
        pairs, rest = [], []
        for l in range(L):
            ws = [self._fused(l, "w")] + [P.c[self._ln(l, n)] for n in self._WT_NAMES]
            for i, (w, t) in enumerate(zip(ws, self._wt[l])):
                if self.blaslt >= 2 and i != 3:
                    continue  # only the dGELU data gradient (FFN2's weight) still reads a copy
                (pairs if self.wt_batch and K.TransposeBatch.fits(w, t) else rest).append((w, t))
        if pairs:
            # every copy in one launch (96 separate launches ran one after another between the
            # forward GEMMs); the pointer table is built once and re-checked per call
            if self._wt_batch is None or len(self._wt_batch.pairs) != len(pairs):
                self._wt_batch = K.TransposeBatch(pairs)
            self._wt_batch.run(pairs)
        for w, t in rest:
            K.krsc_to_crsk(w.view(w.shape[0], 1, 1, w.shape[1]), out=t.view(t.shape[0], 1, 1, t.shape[1]))

    def _inter_buf(self, rows):
        """[rows, intermediate] bf16 activation whose row stride is padded by inter_pad elements
        (a column view of a wider buffer; every GEMM here takes row-strided operands)."""
        I = self.cfg.intermediate_size
        pad = self.inter_pad if self.device.type == "cuda" else 0
        buf = torch.empty((rows, I + pad), dtype=torch.bfloat16, device=self.device)
        return buf[:, :I] if pad else buf

    def _dgrad(self, dy, l, which, **kw):
        """dx = dy · W for encoder weight `which` (0 = fused QKV, 1.. = _WT_NAMES) of layer l."""
        from ..ops import gemm as G
        if self.blaslt >= 2 and set(kw) <= {"out", "beta"}:
            # plain / accumulating data gradients through the vendor library (A/B, TTD_BERT_BLASLT=2)
            w = self._fused(l, "w") if which == 0 else self.params.c[self._ln(l, self._WT_NAMES[which - 1])]
            if kw.get("beta"):
                return kw["out"].addmm_(dy, w)
            return torch.mm(dy, w, out=kw["out"]) if kw.get("out") is not None else torch.mm(dy, w)
        if self._wt is not None and self.transposed_dgrad:
            return G.gemm(dy, self._wt[l][which], trans_b=True, **kw)
        w = self._fused(l, "w") if which == 0 else self.params.c[self._ln(l, self._WT_NAMES[which - 1])]
        return G.gemm(dy, w, **kw)

    def _fused(self, l, what):
        """Zero-copy fused q/k/v views: what in {'w', 'b', 'cb' (bf16 bias), 'gw', 'gb'}."""
        P, H = self.params, self.cfg.hidden_size
        if what in ("w", "gw"):
            o = P.offsets[self._ln(l, "attention/self/query/kernel")]
            buf = P.compute if what == "w" else P.grad
            return buf[o:o + 3 * H * H].view(3 * H, H)
        o = P.offsets[self._ln(l, "attention/self/query/bias")]
        buf = {"b": P.master, "cb": P.compute}.get(what, P.grad)
        return buf[o:o + 3 * H]

    # ------------------------------------------------------------------ training step
    def forward_backward(self, batch: BertBatch, loss_scale: float = 1.0, grad_hook=None):
        """One pre-training forward + backward on the GPU kernels. Gradients of
        loss_scale * (mean MLM loss + mean NSP loss) land in params.grad (loss_scale =
        1/replicas for data parallelism). Returns device fp32[4] =
        (mlm loss, mlm accuracy, nsp loss, nsp accuracy)."""
        from ..ops import gemm as G
        from ..ops import kernels as K
        from ..ops import transformer as T
        c, P = self.cfg, self.params
        dev = self.device
        B, S = batch.input_ids.shape
        H, NH, L = c.hidden_size, c.num_attention_heads, c.num_hidden_layers
        V = c.vocab_size
        Tk = B * S
        hd = c.hidden_dropout_prob if self.dropout else 0.0
        ad = c.attention_probs_dropout_prob if self.dropout else 0.0
        eps = c.layer_norm_eps
        rng = self.rng
        if rng is not None and (hd > 0 or ad > 0):
            rng.advance()
        hook = grad_hook or (lambda name: None)
        bf = torch.bfloat16

        def site(l, k):
            return (l + 1) * 8 + k

        def wgrad(dy, x, out):
            M, N, Kd = dy.shape[1], x.shape[1], dy.shape[0]
            G.gemm(dy, x, trans_a=True, out=out, splits=G.gemm_wgrad_splits(M, N, Kd, big_wgs=self.wgrad_wgs))

        # encoder weight gradients (+ bias column sums) run on a second HIP stream, overlapping
        # the data-gradient chain; the bucket hooks are issued from it so collectives order after
        side = None
        keep = []
        if self.wgrad_stream:
            if getattr(self, "_side", None) is None:
                self._side = torch.cuda.Stream(device=dev)
            side = self._side

        def wgrad_and_bias(dy, x, wout, bout):
            M, N, Kd = dy.shape[1], x.shape[1], dy.shape[0]
            if self.blaslt >= 3:  # A/B: weight gradients through the library too (fp32 output)
                torch.mm(dy.t(), x, out_dtype=torch.float32, out=wout)
                if bout is not None:
                    K.colsum(dy if dy.is_contiguous() else dy.contiguous(), out=bout)
                return
            splits = G.gemm_wgrad_splits(M, N, Kd, big_wgs=self.wgrad_wgs)
            if bout is not None and self.bias_in_wgrad and G.wgrad_bias_ok(M, N, Kd, splits):
                # bias gradient from the weight gradient's own dy tiles (no column-sum pass)
                G.gemm_wgrad_bias(dy, x, wout, bout, splits=splits)
                return
            wgrad(dy, x, wout)
            if bout is not None:
                # (the column-sum kernel reads dense rows: a row-padded dy is compacted first)
                K.colsum(dy if dy.is_contiguous() else dy.contiguous(), out=bout)

        deferred = []

        def wgrad_bias(dy, x, wout, bout, defer=False):
            """weight gradient (+ bias column sum unless bout is None: the producer's epilogue
            already emitted it) on the side stream. defer=True: queued until flush_wgrads(),
            called right after the next LayerNorm backward is enqueued — the side stream then
            starts it only once that LN backward has finished, instead of holding CUs the
            LN backward needs (TTD_BERT_LN_YIELD)."""
            if side is None:
                wgrad_and_bias(dy, x, wout, bout)
                return
            keep.extend((dy, x))  # alive until the streams join (no deferred record_stream frees)
            if defer and self.ln_yield > 0:
                deferred.append((dy, x, wout, bout))
                return
            graphs.fork(torch.cuda.current_stream(), side)
            with torch.cuda.stream(side):
                wgrad_and_bias(dy, x, wout, bout)

        def flush_wgrads():
            if not deferred:
                return
            graphs.fork(torch.cuda.current_stream(), side)
            with torch.cuda.stream(side):
                for a in deferred:
                    if isinstance(a, str):
                        hook(a)  # a gradient-ready hook queued behind the deferred work
                    else:
                        wgrad_and_bias(*a)
            deferred.clear()

        wt_ready = None
        if self.transposed_dgrad:
            if side is not None:  # overlaps the forward pass; the encoder backward waits for it
                graphs.fork(torch.cuda.current_stream(), side)
                with torch.cuda.stream(side):
                    self._refresh_transposed()
                    wt_ready = graphs.mark(side)
            else:
                self._refresh_transposed()

        def layer_hook(name):
            if side is None:
                hook(name)
            elif deferred:
                deferred.append(name)  # after the deferred weight gradients it covers
            else:
                with torch.cuda.stream(side):
                    hook(name)

        ids = batch.input_ids.reshape(-1)
        tt = batch.token_type_ids.reshape(-1)
        seqlen = batch.seqlen
        # MLM rows b*S + positions[b, p] and CLS rows b*S, formed inside the gather / scatter kernels
        pos_idx = batch.masked_lm_positions.reshape(-1)
        if pos_idx.dtype != torch.int32 or not pos_idx.is_contiguous():
            pos_idx = pos_idx.to(torch.int32).contiguous()
        pos_grp = (batch.masked_lm_positions.shape[1], S)
        labels = batch.masked_lm_ids.reshape(-1).contiguous()

        # ---------------------------------------------------------------- forward
        s0 = T.embed_fwd(ids, tt, P.c["bert/embeddings/word_embeddings"], P.c["bert/embeddings/position_embeddings"],
                         P.c["bert/embeddings/token_type_embeddings"], S)
        y, _, mean0, rstd0 = T.layernorm_fwd(s0, P.var["bert/embeddings/LayerNorm/gamma"],
                                             P.var["bert/embeddings/LayerNorm/beta"], eps=eps, p_out=hd,
                                             site_out=1, rng=rng)
        ctx = []
        for l in range(L):
            x = y
            qkv = self._plain(x, self._fused(l, "w"), self._fused(l, "b"), self._fused(l, "cb"))
            ao = torch.empty((Tk, H), dtype=bf, device=dev)
            lse = torch.empty((B * NH, S), dtype=torch.float32, device=dev)
            T.attention_fwd(qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], ao, lse, B, NH, S, seqlen=seqlen,
                            p_drop=ad, rng=rng, site=site(l, 0))
            nb = self._ln(l, "attention/output/dense/bias")
            proj = self._plain(ao, P.c[self._ln(l, "attention/output/dense/kernel")], P.var[nb], P.c[nb])
            y1, s1, m1, r1 = T.layernorm_fwd(proj, P.var[self._ln(l, "attention/output/LayerNorm/gamma")],
                                             P.var[self._ln(l, "attention/output/LayerNorm/beta")], res=x, eps=eps,
                                             p_in=hd, site_in=site(l, 1), rng=rng)
            del proj
            pre = self._inter_buf(Tk)
            inter = G.gemm(y1, P.c[self._ln(l, "intermediate/dense/kernel")], trans_b=True, out=self._inter_buf(Tk),
                           bias=P.var[self._ln(l, "intermediate/dense/bias")], act=G.ACT_GELU, aux=pre)
            nb = self._ln(l, "output/dense/bias")
            o2 = self._plain(inter, P.c[self._ln(l, "output/dense/kernel")], P.var[nb], P.c[nb])
            y, s2, m2, r2 = T.layernorm_fwd(o2, P.var[self._ln(l, "output/LayerNorm/gamma")],
                                            P.var[self._ln(l, "output/LayerNorm/beta")], res=y1, eps=eps, p_in=hd,
                                            site_in=site(l, 2), rng=rng)
            del o2
            ctx.append((x, qkv, ao, lse, s1, m1, r1, y1, pre, inter, s2, m2, r2))

        # masked-LM head
        hm = T.gather_rows(y, pos_idx, group=pos_grp)
        tpre = torch.empty_like(hm)
        t = G.gemm(hm, P.c["cls/predictions/transform/dense/kernel"], trans_b=True,
                   bias=P.var["cls/predictions/transform/dense/bias"], act=G.ACT_GELU, aux=tpre)
        t2, _, mt, rt = T.layernorm_fwd(t, P.var["cls/predictions/transform/LayerNorm/gamma"],
                                        P.var["cls/predictions/transform/LayerNorm/beta"], eps=eps)
        logits = self._plain(t2, P.c["bert/embeddings/word_embeddings"], P.var["cls/predictions/output_bias"],
                             P.c["cls/predictions/output_bias"])
        sums = K.zeros(4, dtype=torch.float32, device=dev)  # own memset: no torch fill kernel in the step
        cnt = T.count_valid2(labels, loss_scale, torch.empty(2, dtype=torch.float32, device=dev))
        inv_cnt, gsc = cnt[0:1], cnt[1:2]  # metric scale 1 / count, gradient scale loss_scale / count
        T.xent_vocab(logits, V, labels, gsc, dlogits=logits, sums=sums[0:2], mscale=inv_cnt)
        dlog = logits  # gradient now, in place
        # next-sentence head
        cls = T.gather_rows(y, None, group=(1, S), n=B)
        pooled = G.gemm(cls, P.c["bert/pooler/dense/kernel"], trans_b=True, bias=P.var["bert/pooler/dense/bias"],
                        act=G.ACT_TANH)
        nsp = G.gemm(pooled, P.c["cls/seq_relationship/output_weights"], trans_b=True,
                     bias=P.var["cls/seq_relationship/output_bias"])
        nsums, dnsp, _, _ = K.sparse_xent(nsp, batch.next_sentence_labels, grad_scale=loss_scale / B)
        sums[2:4].copy_(nsums)

        # ---------------------------------------------------------------- backward: heads
        g = P.g
        wgrad(dlog, t2, g["bert/embeddings/word_embeddings"])  # tied decoder (write; embedding adds later)
        K.colsum(dlog, out=g["cls/predictions/output_bias"])
        hook("cls/predictions/output_bias")
        dt2 = (torch.mm(dlog, P.c["bert/embeddings/word_embeddings"]) if self.blaslt >= 2
               else G.gemm(dlog, P.c["bert/embeddings/word_embeddings"]))
        del dlog, logits
        dt, _ = T.layernorm_bwd(dt2, t, mt, rt, P.var["cls/predictions/transform/LayerNorm/gamma"],
                                g["cls/predictions/transform/LayerNorm/gamma"],
                                g["cls/predictions/transform/LayerNorm/beta"])
        hook("cls/predictions/transform/LayerNorm/beta")
        dtp = T.dact(dt, tpre, 0)
        wgrad(dtp, hm, g["cls/predictions/transform/dense/kernel"])
        K.colsum(dtp, out=g["cls/predictions/transform/dense/bias"])
        dhm = G.gemm(dtp, P.c["cls/predictions/transform/dense/kernel"])
        hook("cls/predictions/transform/dense/bias")
        wgrad(dnsp, pooled, g["cls/seq_relationship/output_weights"])
        K.colsum(dnsp, out=g["cls/seq_relationship/output_bias"])
        dpooled = G.gemm(dnsp, P.c["cls/seq_relationship/output_weights"])
        hook("cls/seq_relationship/output_bias")
        dpp = T.dact(dpooled, pooled, 1)
        wgrad(dpp, cls, g["bert/pooler/dense/kernel"])
        K.colsum(dpp, out=g["bert/pooler/dense/bias"])
        dcls = G.gemm(dpp, P.c["bert/pooler/dense/kernel"])
        hook("bert/pooler/dense/bias")
        dy = K.zeros((Tk, H), dtype=bf, device=dev)
        T.scatter_rows(dhm, pos_idx, dy, group=pos_grp)
        T.scatter_rows(dcls, None, dy, accumulate=True, group=(1, S))

        # ---------------------------------------------------------------- backward: encoder
        ln_work = T.ln_bwd_workspace(Tk, H, dev)
        # FFN1 bias gradient from the FFN2-dgrad epilogue statistics (256-row GEMM tiles)
        fuse_bias = self.fuse_bias_grad and G.big_fits(Tk, c.intermediate_size, H)
        bias_part = (torch.empty((-(-Tk // 256), 2, c.intermediate_size), dtype=torch.float32, device=dev)
                     if fuse_bias else None)
        delta = torch.empty((B * NH, S), dtype=torch.float32, device=dev)
        if wt_ready is not None:
            graphs.join_mark(torch.cuda.current_stream(), wt_ready)
        for l in reversed(range(L)):
            x, qkv, ao, lse, s1, m1, r1, y1, pre, inter, s2, m2, r2 = ctx.pop()
            G1 = torch.empty((Tk, H), dtype=bf, device=dev)
            _, dout2 = T.layernorm_bwd(dy, s2, m2, r2, P.var[self._ln(l, "output/LayerNorm/gamma")],
                                       g[self._ln(l, "output/LayerNorm/gamma")],
                                       g[self._ln(l, "output/LayerNorm/beta")], ds_out=G1, want_dx=True, p_in=hd,
                                       site_in=site(l, 2), rng=rng, work=ln_work)
            flush_wgrads()
            del dy
            wgrad_bias(dout2, inter, g[self._ln(l, "output/dense/kernel")], g[self._ln(l, "output/dense/bias")])
            b_inter = g[self._ln(l, "intermediate/dense/bias")]
            if fuse_bias:
                # the intermediate bias gradient = column sums of dpre, taken from the per-tile
                # statistics of the dGELU dgrad epilogue that produces dpre (no separate column-sum
                # pass over the [tokens, 4096] gradient)
                dpre = self._dgrad(dout2, l, 3, act=G.ACT_DGELU, residual=pre, stat=bias_part, tile=(256, 0),
                                   out=self._inter_buf(Tk))
                K.col_reduce2(bias_part, bias_part.shape[0], o0=b_inter)
                b_inter = None
            else:
                dpre = self._dgrad(dout2, l, 3, act=G.ACT_DGELU, residual=pre, out=self._inter_buf(Tk))
            del dout2, inter, pre
            wgrad_bias(dpre, y1, g[self._ln(l, "intermediate/dense/kernel")], b_inter, defer=True)
            self._dgrad(dpre, l, 2, out=G1, beta=1)
            del dpre
            layer_hook(self._ln(l, "intermediate/dense/bias"))
            G0 = torch.empty((Tk, H), dtype=bf, device=dev)
            _, dproj = T.layernorm_bwd(G1, s1, m1, r1, P.var[self._ln(l, "attention/output/LayerNorm/gamma")],
                                       g[self._ln(l, "attention/output/LayerNorm/gamma")],
                                       g[self._ln(l, "attention/output/LayerNorm/beta")], ds_out=G0, want_dx=True,
                                       p_in=hd, site_in=site(l, 1), rng=rng, work=ln_work)
            if self.ln_yield != 2:
                flush_wgrads()
            del G1
            wgrad_bias(dproj, ao, g[self._ln(l, "attention/output/dense/kernel")],
                       g[self._ln(l, "attention/output/dense/bias")], defer=self.ln_yield == 2)
            dao = self._dgrad(dproj, l, 1)
            del dproj
            dqkv = torch.empty((Tk, 3 * H), dtype=bf, device=dev)
            T.attention_bwd(qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], ao, dao, lse, dqkv[:, :H],
                            dqkv[:, H:2 * H], dqkv[:, 2 * H:], B, NH, S, delta=delta, seqlen=seqlen, p_drop=ad,
                            rng=rng, site=site(l, 0))
            if self.ln_yield == 2:
                flush_wgrads()  # (mode 2: the attention backward runs without side-stream GEMMs too)
            del dao, ao, qkv
            wgrad_bias(dqkv, x, self._fused(l, "gw"), self._fused(l, "gb"), defer=l > 0)
            self._dgrad(dqkv, l, 0, out=G0, beta=1)
            del dqkv
            layer_hook(self._ln(l, "attention/self/value/bias"))
            dy = G0
        if side is not None:
            flush_wgrads()
            graphs.join(torch.cuda.current_stream(), side)
        keep.clear()

        # ---------------------------------------------------------------- backward: embeddings
        ds0, _ = T.layernorm_bwd(dy, s0, mean0, rstd0, P.var["bert/embeddings/LayerNorm/gamma"],
                                 g["bert/embeddings/LayerNorm/gamma"], g["bert/embeddings/LayerNorm/beta"], p_out=hd,
                                 site_out=1, rng=rng, work=ln_work)
        dpos = g["bert/embeddings/position_embeddings"]
        if S < dpos.shape[0]:
            K.zero_(dpos[S:])
        T.embed_bwd(ds0, ids, tt, g["bert/embeddings/word_embeddings"], dpos, g["bert/embeddings/token_type_embeddings"],
                    B, S)
        hook("bert/embeddings/word_embeddings")
        return sums

    # ------------------------------------------------------------------ fp32 reference (tests)
    def reference_loss(self, batch: BertBatch, leaves: dict):
        """Plain-PyTorch fp32 forward (dropout off) on `leaves` (name -> fp32 tensor with
        requires_grad as wanted). Returns (mlm mean loss, nsp mean loss)."""
        import torch.nn.functional as F
        c = self.cfg
        H, NH, L, V = c.hidden_size, c.num_attention_heads, c.num_hidden_layers, c.vocab_size
        B, S = batch.input_ids.shape
        W = leaves

        def lin(x, name):
            return x @ W[name + "/kernel"].t() + W[name + "/bias"]

        def ln(x, name):
            return F.layer_norm(x, (H,), W[name + "/gamma"], W[name + "/beta"], c.layer_norm_eps)

        def gelu(x):
            return 0.5 * x * (1 + torch.tanh(0.7978845608028654 * (x + 0.044715 * x ** 3)))

        ids = batch.input_ids.long()
        x = (W["bert/embeddings/word_embeddings"][ids] + W["bert/embeddings/position_embeddings"][:S][None]
             + W["bert/embeddings/token_type_embeddings"][batch.token_type_ids.long()])
        x = ln(x, "bert/embeddings/LayerNorm")
        keymask = None
        if batch.seqlen is not None:
            ar = torch.arange(S, device=x.device)
            keymask = ar[None, :] < batch.seqlen[:, None].long()
        for l in range(L):
            p = lambda s, l=l: self._ln(l, s)  # noqa: E731
            q = lin(x, p("attention/self/query")).view(B, S, NH, 64).transpose(1, 2)
            k = lin(x, p("attention/self/key")).view(B, S, NH, 64).transpose(1, 2)
            v = lin(x, p("attention/self/value")).view(B, S, NH, 64).transpose(1, 2)
            sc = q @ k.transpose(-1, -2) / 8.0
            if keymask is not None:
                sc = sc.masked_fill(~keymask[:, None, None, :], float("-inf"))
            a = (sc.softmax(-1) @ v).transpose(1, 2).reshape(B, S, H)
            x = ln(x + lin(a, p("attention/output/dense")), p("attention/output/LayerNorm"))
            h = gelu(lin(x, p("intermediate/dense")))
            x = ln(x + lin(h, p("output/dense")), p("output/LayerNorm"))
        flat = x.reshape(B * S, H)
        offs = torch.arange(B, device=x.device) * S
        pos = (batch.masked_lm_positions.long() + offs[:, None]).reshape(-1)
        t = ln(gelu(lin(flat[pos], "cls/predictions/transform/dense")), "cls/predictions/transform/LayerNorm")
        logits = t @ W["bert/embeddings/word_embeddings"][:V].t() + W["cls/predictions/output_bias"][:V]
        lab = batch.masked_lm_ids.reshape(-1).long()
        mlm = F.cross_entropy(logits, lab.clamp(min=0), reduction="none")
        valid = (lab >= 0).float()
        mlm = (mlm * valid).sum() / valid.sum().clamp(min=1)
        pooled = torch.tanh(lin(flat[offs], "bert/pooler/dense"))
        nl = pooled @ W["cls/seq_relationship/output_weights"].t() + W["cls/seq_relationship/output_bias"]
        nsp = F.cross_entropy(nl, batch.next_sentence_labels.long())
        return mlm, nsp


def bert_large(device="cuda", **kw) -> BertPretraining:
    return BertPretraining(BertConfig.large(), device=device, **kw)
